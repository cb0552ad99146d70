#!/bin/bash
# One development round trip on the GPU box: selection self-check, GPU parity tests, the
# default bench line (no CPU baseline) and a rocprofv3 kernel trace of it with its
# per-run timeline.  Stops at the first failing GPU step.  usage: tools/iter.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-iter}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ -z "$SKIP_SELCHECK" ]; then
    bash tools/selcheck.sh > "$out/selcheck.log" 2>&1 || { echo "selcheck failed"; tail -20 "$out/selcheck.log"; exit 1; }
    grep -E "^n=|total" "$out/selcheck.log"
fi
if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
    rc=$?; tail -5 "$out/pytest_gpu.log"
    [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > "$out/bench.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$out/bench.log"; exit 1; }
tail -1 "$out/bench.log" | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --no-cpu-baseline --sustain-s 0 ${BENCH_ARGS} > "$out/bench_rocprof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
python3 tools/timeline.py "$out/prof/run_kernel_trace.csv" > "$out/timeline.txt" 2>&1
cat "$out/timeline.txt" | head -30
