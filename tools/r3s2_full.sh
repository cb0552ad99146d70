#!/bin/bash
# Round-3 (session 2): the whole GPU suite, smoke and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/r3s2_full
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$out/pytest_gpu.log"
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke failed"; tail "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 600 python bench.py > "$out/bench.log" 2>&1 || { echo "bench failed"; tail "$out/bench.log"; exit 1; }
tail -1 "$out/bench.log" | cut -c1-600
