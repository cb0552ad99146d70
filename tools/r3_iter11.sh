#!/bin/bash
# Round-3 iteration 11: parity (DPP block reductions, pair prefetch from the gather,
# k_nn_grid_q from the 5th call), then C3 A/B of the call index where k_nn_grid_q starts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it11
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_ties_golden.py tests/test_gpu_configs.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 700 bash tools/ab_bench.sh FICP_NN_QPT_FROM=1000 FICP_NN_QPT_FROM=3 FICP_NN_QPT_FROM=6 || exit 1
