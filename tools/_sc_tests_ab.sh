#!/bin/bash
# selcheck over all modes, the GPU tests, then ab_bench against the given variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
bash tools/selcheck.sh > gpurun_out/sc.log 2>&1 || { echo "selcheck failed"; tail -5 gpurun_out/sc.log; exit 1; }
echo "selcheck ok: $(grep -c 'bad=0' gpurun_out/sc.log) configs"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
bash tools/ab_bench.sh "$@"
