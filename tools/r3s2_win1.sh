#!/bin/bash
# Round-3 (session 2) iteration 1: the one-launch window selection (k_sel_win).
# Window tests, the C3 configs and the parity suite's run tests, then an A/B of the bench
# with the window path on / off and a rocprof timeline of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/r3s2_win1
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py -x -v --timeout 300 --timeout-method thread > "$out/pytest_win.log" 2>&1
rc=$?; tail -15 "$out/pytest_win.log"
[ $rc -ne 0 ] && { echo "window tests rc=$rc"; exit $rc; }
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 400 bash tools/ab_bench.sh FICP_SEL_WIN=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --no-cpu-baseline --no-extra --steps 10 --warmup 2 > "$out/bench_rocprof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
python3 tools/timeline.py "$out/prof/run_kernel_trace.csv" > "$out/timeline.txt" 2>&1
head -80 "$out/timeline.txt"
