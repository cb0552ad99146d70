#!/bin/bash
# Round-3 iteration 5: batch parity (two sub-batch streams), then the shares with one and
# two streams, and a timeline of the 128-plot share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it5
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_batch.py > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
for rep in 1 2; do
for p in 128 256 512; do
  for ns in 1 2; do
    FICP_BATCH_STREAMS=$ns timeout -k 10 120 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b${p}_s$ns.log" 2>&1 || { echo "batch $p failed"; tail -5 "$out/b${p}_s$ns.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/b${p}_s$ns.log').read().strip().splitlines()[-1]); print('plots $p streams $ns', round(d['value']), round(d['ms_per_step'],3))"
  done
done
done
timeout -k 10 120 python bench.py --workload batch --plots 1024 --steps 10 --warmup 2 --no-cpu-baseline > "$out/b1024.log" 2>&1 || { echo "batch 1024 failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$out/b1024.log').read().strip().splitlines()[-1]); print('plots 1024', round(d['value']), round(d['ms_per_step'],3))"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof128" -o run -- \
    python3 bench.py --workload batch --plots 128 --steps 3 --warmup 1 --no-cpu-baseline > "$out/prof128.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/timeline.py "$out/prof128/run_kernel_trace.csv" k_batch_init > "$out/timeline128.txt" 2>&1
head -16 "$out/timeline128.txt"
