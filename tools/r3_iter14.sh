#!/bin/bash
# Round-3 iteration 14: batch parity with the live count folded into the selection, and
# the shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it14
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
for rep in 1 2; do
  for p in 128 256 1024; do
    timeout -k 10 150 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b$p.log" 2>&1 || { echo "batch $p failed"; tail -5 "$out/b$p.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/b$p.log').read().strip().splitlines()[-1]); print('plots $p', round(d['value']), round(d['ms_per_step'],3))"
  done
done
