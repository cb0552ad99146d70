#!/bin/bash
# Round-3 (session 2): the batch window path -- batch parity tests, then the 128- and
# 1024-plot bench lines with the path on / off (FICP_BSEL_WIN=0), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/r3s2_batch2
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > "$out/pytest_batch.log" 2>&1
rc=$?; tail -3 "$out/pytest_batch.log"
[ $rc -ne 0 ] && { echo "batch tests rc=$rc"; exit $rc; }
for rep in 1 2; do
for P in 128 1024; do
for W in 1 0; do
  FICP_BSEL_WIN=$W timeout -k 10 300 python3 bench.py --workload batch --plots $P --no-cpu-baseline --no-extra --steps 10 --warmup 2 > "$out/bench_${P}_$W.log" 2>&1 || { echo "bench $P failed"; tail "$out/bench_${P}_$W.log"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$out/bench_${P}_$W.log').read().strip().splitlines()[-1]); print('plots $P win $W', round(d['value']), d['unit'], round(d['ms_per_step'],3), 'ms')"
done; done; done
