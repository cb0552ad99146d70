#!/bin/bash
# Round-3 iteration 20: parity with the DPP range and block min/max reductions, A/B against HEAD (prev)
#
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it21
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_ties_golden.py tests/test_gpu_configs.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
BENCH_ARGS="--no-extra --steps 60 --warmup 5" timeout -k 10 600 bash tools/ab_bench.sh prev || exit 1
