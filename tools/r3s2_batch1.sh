#!/bin/bash
# Round-3 (session 2): the batch workload at the N = 8 per-rank share (128 plots) and the
# N = 1 batch (1024 plots): bench lines and a rocprof timeline of the 128-plot run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/r3s2_batch1
mkdir -p "$out"
for P in 128 1024; do
  timeout -k 10 300 python3 bench.py --workload batch --plots $P --no-cpu-baseline --no-extra --steps 10 --warmup 2 > "$out/bench_$P.log" 2>&1 || { echo "bench $P failed"; tail "$out/bench_$P.log"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$out/bench_$P.log').read().strip().splitlines()[-1]); print($P, round(d['value']), d['unit'], round(d['ms_per_step'],3), 'ms')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --workload batch --plots 128 --no-cpu-baseline --no-extra --steps 4 --warmup 1 > "$out/bench_rocprof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
head -25 "$out/prof/run_kernel_stats.csv" | cut -d, -f1-8
