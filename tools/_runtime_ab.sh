#!/bin/bash
# A/B of the HIP runtime libficp.so binds to (torch's bundled one vs /opt/rocm's), then
# the C5 config test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_torch_$i.log 2>&1 || exit $?
  FICP_HIP_RUNTIME=system timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_system_$i.log 2>&1 || exit $?
done
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 800 --timeout-method thread -k c5 > gpurun_out/c5.log 2>&1
rc=$?
tail -5 gpurun_out/c5.log
exit $rc
