#!/bin/bash
# kernel trace of a short bench: gpurun_out/tr/<name>; usage: tools/_trace_run.sh name [NAME=VALUE ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
name=$1; shift
out=gpurun_out/tr/$name
mkdir -p "$out"
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > "$out/bench.log" 2>&1 || exit $?
find "$out/prof" -name '*kernel_trace.csv' -exec cp {} "$out/trace.csv" \;
rm -rf "$out/prof"
