#!/bin/bash
# Round-3 (session 2) iteration 2: window path phase stamps (FICP_WIN_PROF variant), the
# window tests, and an A/B of the bench with the window path on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/r3s2_win2
mkdir -p "$out"
FICP_LIB=$PWD/tools/ab/libficp_winprof.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extra --steps 3 --warmup 1 > "$out/winprof.log" 2>&1 || { echo "winprof failed"; tail "$out/winprof.log"; exit 1; }
grep WINPROF "$out/winprof.log" | tail -10
timeout -k 10 400 python -u -m pytest tests/test_gpu_window.py -x -q --timeout 300 --timeout-method thread > "$out/pytest_win.log" 2>&1
rc=$?; tail -3 "$out/pytest_win.log"
[ $rc -ne 0 ] && { echo "window tests rc=$rc"; exit $rc; }
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 400 bash tools/ab_bench.sh FICP_SEL_WIN=0 || exit 1
