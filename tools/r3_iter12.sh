#!/bin/bash
# Round-3 iteration 12: batch parity (DPP block reductions, four sub-batch streams), the
# shares with 2 vs 4 streams, and the C3 selection phase stamps (SEL_PROF build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it12
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
run() {  # plots, label, env...
  local p=$1 lab=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b${p}_$lab.log" 2>&1 || { echo "batch $p $lab failed"; tail -5 "$out/b${p}_$lab.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/b${p}_$lab.log').read().strip().splitlines()[-1]); print('plots $p $lab', round(d['value']), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  for p in 128 256; do
    run $p s2 FICP_BATCH_STREAMS=2 || exit 1
    run $p s3 FICP_BATCH_STREAMS=3 || exit 1
    run $p s4 FICP_BATCH_STREAMS=4 || exit 1
  done
done
run 1024 s2 FICP_BATCH_STREAMS=2 || exit 1
run 1024 s4 FICP_BATCH_STREAMS=4 || exit 1
FICP_LIB=$PWD/tools/ab/libficp_selprof.so timeout -k 10 120 python bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 1 > "$out/selprof.log" 2>&1 || { echo "selprof failed"; tail -5 "$out/selprof.log"; exit 1; }
grep SELPROF "$out/selprof.log" | head -6
