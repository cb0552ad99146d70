#!/bin/bash
# Round-3 iteration 13: parity with the one-round block bounds, C3 A/B against the
# one-workgroup bounds (FICP_SEL_RB=0), the phase stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it13
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_ties_golden.py tests/test_gpu_configs.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 400 bash tools/ab_bench.sh FICP_SEL_RB=0 || exit 1
FICP_LIB=$PWD/tools/ab/libficp_selprof.so timeout -k 10 120 python bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 1 > "$out/selprof.log" 2>&1 || { echo "selprof failed"; tail -5 "$out/selprof.log"; exit 1; }
grep SELPROF "$out/selprof.log" | head -4
