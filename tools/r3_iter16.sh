#!/bin/bash
# Round-3 iteration 16: longer C3 A/B of the remaining defaults (stored vs derived sort
# keys, the first k_nn_grid_q call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
BENCH_ARGS="--no-extra --steps 80 --warmup 5" timeout -k 10 900 bash tools/ab_bench.sh FICP_NN_KEYS=1 FICP_NN_QPT_FROM=3 FICP_NN_QPT_FROM=5 || exit 1
