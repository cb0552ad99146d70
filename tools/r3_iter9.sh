#!/bin/bash
# Round-3 iteration 9: run-to-run determinism (md2/md3 probes), batch parity + shares with
# the fixed-point bucket sums, and the NN per-call counters (FICP_NN_STATS build) at C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it9
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python tools/md2_probe2.py 2 no || exit 1
FICP_FUSE_FIT=0 timeout -k 10 120 python tools/md2_probe2.py 2 no || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
for p in 128 1024; do
  timeout -k 10 150 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b$p.log" 2>&1 || { echo "batch $p failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/b$p.log').read().strip().splitlines()[-1]); print('plots $p', round(d['value']), round(d['ms_per_step'],3))"
done
FICP_LIB=$PWD/tools/ab/libficp_nnstats.so timeout -k 10 120 python bench.py --no-extra --no-cpu-baseline --steps 2 --warmup 1 > "$out/nnstats.log" 2>&1 || { echo "nnstats failed"; tail -5 "$out/nnstats.log"; exit 1; }
grep NNSTATS "$out/nnstats.log" | tail -14
