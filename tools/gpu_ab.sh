#!/bin/bash
# GPU parity tests, then the C3 bench with the bucketed selection (default) and with the
# full residual sort (FICP_SELECT=0); stops at the first failure of a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_sel.log 2>&1 || { echo "bench(select) rc=$?"; tail -20 gpurun_out/bench_sel.log; exit 1; }
tail -1 gpurun_out/bench_sel.log
FICP_SELECT=0 timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_sort.log 2>&1 || { echo "bench(sort) rc=$?"; exit 1; }
tail -1 gpurun_out/bench_sort.log
