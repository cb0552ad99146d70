#!/bin/bash
# Round-3 iteration 17: batch parity and the shares with the sub-batches' start staggered
# by one NN (FICP_BATCH_STAGGER=0: lockstep), plus a timeline of the 128-plot share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it17
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
run() {  # plots, label, env...
  local p=$1 lab=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b${p}_$lab.log" 2>&1 || { echo "batch $p $lab failed"; tail -5 "$out/b${p}_$lab.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/b${p}_$lab.log').read().strip().splitlines()[-1]); print('plots $p $lab', round(d['value']), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  for p in 128 256 1024; do
    run $p stag FICP_BATCH_STAGGER=1 || exit 1
    run $p lock FICP_BATCH_STAGGER=0 || exit 1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof128" -o run -- \
    python3 bench.py --workload batch --plots 128 --steps 3 --warmup 1 --no-cpu-baseline > "$out/prof128.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/timeline.py "$out/prof128/run_kernel_trace.csv" k_batch_init -v > "$out/timeline128.txt" 2>&1
sed -n 1,40p "$out/timeline128.txt"
