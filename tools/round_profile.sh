#!/bin/bash
# The default bench line and the rocprofv3 kernel summary of the same command, for
# profiles/<tag>_*: usage tools/round_profile.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r1}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 bench.py > "$out/bench.log" 2>&1 || exit $?
grep '^{' "$out/bench.log" | tail -1 > "$out/bench.json"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py > "$out/bench_under_rocprof.log" 2>&1 || exit $?
find "$out/prof" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
cat "$out/bench.json"
