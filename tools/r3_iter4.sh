#!/bin/bash
# Round-3 iteration 4: batch parity with the device-planned grids, then the shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it4
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_batch.py tests/test_gpu_errors.py > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
for p in 1024 128; do
  for hp in 0 1; do
    if [ $hp = 1 ]; then export FICP_BATCH_HOSTPLAN=1; else unset FICP_BATCH_HOSTPLAN; fi
    timeout -k 10 120 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b${p}_h$hp.log" 2>&1 || { echo "batch $p failed"; tail -5 "$out/b${p}_h$hp.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/b${p}_h$hp.log').read().strip().splitlines()[-1]); print('plots $p hostplan $hp', round(d['value']), round(d['ms_per_step'],3), {k:round(v['ms'],3) for k,v in d['kernel_ms'].items()})"
  done
done
unset FICP_BATCH_HOSTPLAN
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof128" -o run -- \
    python3 bench.py --workload batch --plots 128 --steps 3 --warmup 1 --no-cpu-baseline > "$out/prof128.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/timeline.py "$out/prof128/run_kernel_trace.csv" k_batch_init > "$out/timeline128.txt" 2>&1
head -16 "$out/timeline128.txt"
