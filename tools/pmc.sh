#!/bin/bash
# PMC passes of the bench (one counter group per rocprofv3 run, as MI355X_MICROARCH.md
# prescribes: FETCH_SIZE and WRITE_SIZE cannot share a pass).  No trace domains.
# usage: tools/pmc.sh <name> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
name=${1:-pmc}; shift
out=gpurun_out/$name
mkdir -p "$out"
export TMPDIR=/tmp
i=0
groups=${PMC_GROUPS:-"FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
IFS='|' read -ra GROUPS_ARR <<< "$groups"
for ctr in "${GROUPS_ARR[@]}"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$out/p$i" -o run -- \
        python3 bench.py --no-cpu-baseline --sustain-s 0 --steps 2 --warmup 1 "$@" > "$out/p$i.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$out" > "$out/summary.json"
cat "$out/summary.json"
