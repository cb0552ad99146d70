#!/bin/bash
# rocprofv3 kernel-trace + stats of the default bench command (CSV output).
# usage: tools/profile.sh <outdir-name> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
name=${1:-prof}; shift
out=gpurun_out/$name
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
    python3 bench.py --no-cpu-baseline --sustain-s 0 "$@" > "$out/bench.log" 2>&1
rc=$?
grep '^{' "$out/bench.log" | tail -1
find "$out" -name '*kernel_stats.csv' -exec head -30 {} \;
exit $rc
