#!/bin/bash
# A/B of variants (tools/ab_bench.sh) then a kernel-trace timeline of the default library.
# usage: tools/_ab_trace.sh <tag> variant...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=$1; shift
export TMPDIR=/tmp
bash tools/ab_bench.sh "$@" || exit $?
out=gpurun_out/$tag
mkdir -p "$out"
[ -n "$TRACE_LIB" ] && export FICP_LIB=$PWD/tools/ab/libficp_$TRACE_LIB.so
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --no-cpu-baseline --no-extra --steps 5 --warmup 2 > "$out/bench_rocprof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
python3 tools/timeline.py "$out/prof/run_kernel_trace.csv" k_minmax2_partial -v > "$out/timeline_v.txt" 2>&1
rm -f "$out"/prof/*.db
tail -22 "$out/timeline_v.txt"
