#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Stops at the first GPU fault,
# abort or timeout (exit codes other than 0/1 from pytest).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
rc=0
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
cat gpurun_out/smoke.log | tail -5
if [ $src -ne 0 ] && [ $src -ne 1 ]; then echo "smoke rc=$src: stopping"; exit $src; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
echo "pytest=$rc smoke=$src bench=$brc"
