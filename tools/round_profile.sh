#!/bin/bash
# The default bench line (with its CPU baseline), the rocprofv3 kernel trace + stats of
# the same command, and the PMC passes of the NN kernel (tools/pmc.sh), all under
# gpurun_out/<tag>/.  tools/make_profiles.py <tag> turns them into profiles/r1_*.
# usage: tools/round_profile.sh <tag>
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
bash tools/pmc.sh "$tag/pmc" > "$out/pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "$out/pmc.log"; exit 1; }
cat "$out/bench.json"
