#!/bin/bash
# The non-headline bench workloads (C2, C4 batch, C5 partitioned on one GPU), one line each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/wl
for w in c2 batch c5; do
  extra=""; [ $w = c5 ] && extra="--local-shards 8"  # C5 as DESIGN §7 quotes it: 8 local ranks
  timeout -k 10 400 python bench.py --no-cpu-baseline --workload $w $extra > gpurun_out/wl/$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/wl/$w.log; exit 1; }
  tail -1 gpurun_out/wl/$w.log | cut -c1-600
done
