#!/bin/bash
# Round-3 iteration 10: parity with the bounds spread over the reduce (k_sel_reduce_bounds)
# and 4 queries per NN thread; C3 A/B of NN variants and of the old bounds; a timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it10
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_ties_golden.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 700 bash tools/ab_bench.sh nnold q4w6 q2w6 q2w5 FICP_SEL_RB=0 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --no-extra --no-cpu-baseline --steps 4 --warmup 1 > "$out/prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/timeline.py "$out/prof/run_kernel_trace.csv" k_run_start -v > "$out/timeline.txt" 2>&1
tail -16 "$out/timeline.txt"
grep -E "k_nn_grid|k_sel" "$out/timeline.txt" | head -30
