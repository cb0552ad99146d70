#!/bin/bash
# Round-3 iteration 6: batch parity with the loop step + fit fused into the selection, then
# the shares: fused vs separate launches, one vs two streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it6
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_batch.py > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
run() {  # plots, label, env...
  local p=$1 lab=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b${p}_$lab.log" 2>&1 || { echo "batch $p $lab failed"; tail -5 "$out/b${p}_$lab.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/b${p}_$lab.log').read().strip().splitlines()[-1]); print('plots $p $lab', round(d['value']), round(d['ms_per_step'],3), {k:round(v['ms'],3) for k,v in d['kernel_ms'].items()})"
}
for rep in 1 2; do
  run 128 fused FICP_BATCH_FUSE=1 || exit 1
  run 128 sep FICP_BATCH_FUSE=0 || exit 1
  run 1024 fused_s1 FICP_BATCH_FUSE=1 FICP_BATCH_STREAMS=1 || exit 1
  run 1024 fused_s2 FICP_BATCH_FUSE=1 FICP_BATCH_STREAMS=2 || exit 1
  run 1024 sep_s1 FICP_BATCH_FUSE=0 FICP_BATCH_STREAMS=1 || exit 1
done
run 128 fused_s1 FICP_BATCH_STREAMS=1 || exit 1
run 512 fused_s2 FICP_BATCH_STREAMS=2 || exit 1
run 512 fused_s1 FICP_BATCH_STREAMS=1 || exit 1
