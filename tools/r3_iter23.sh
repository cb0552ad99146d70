#!/bin/bash
# Round-3 iteration 23: C3 A/B of the histogram's shape (8 rows in flight per thread; 256
# workgroups of 4096 rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
BENCH_ARGS="--no-extra --steps 60 --warmup 5" timeout -k 10 600 bash tools/ab_bench.sh hu8 hb256 || exit 1
