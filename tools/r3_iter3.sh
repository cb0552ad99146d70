#!/bin/bash
# Round-3 iteration 3: parity of the new paths (small plots, wide batch selection, split
# selection, prefetching final), batch-share A/B of the wide selection, fused-fit A/B at C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it3
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_errors.py tests/test_ties_golden.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
for rep in 1 2; do
  for p in 128 256; do
    for w in 0 1; do
      FICP_BSEL_WIDE=$w timeout -k 10 120 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b${p}_w$w.log" 2>&1 || { echo "batch $p w$w failed"; tail -5 "$out/b${p}_w$w.log"; exit 1; }
      python3 -c "import json; d=json.loads(open('$out/b${p}_w$w.log').read().strip().splitlines()[-1]); print('plots $p wide $w', round(d['value']), round(d['ms_per_step'],3), {k:round(v['ms'],3) for k,v in d['kernel_ms'].items()})"
    done
  done
done
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 400 bash tools/ab_bench.sh FICP_FUSE_FIT=0 || exit 1
