#!/bin/bash
# The default bench line (with its CPU baseline), the rocprofv3 kernel trace + stats of
# the same command, the PMC passes of the NN kernel (tools/pmc.sh) with the 8-B-per-lane
# FETCH/WRITE calibration (tools/pmc_calib.py), and the drop-in call under a HIP API
# trace (tools/host_path_trace.py), all under gpurun_out/<tag>/.
# tools/make_profiles.py <tag> <prefix> turns them into profiles/<prefix>_*, and
# tools/make_batch_pmc.py gpurun_out/<tag>/pmc_batch <prefix> the batch NN's PMC bytes.
# usage: tools/round_profile.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r3}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 bench.py > "$out/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" | tail -1 > "$out/bench.json"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --no-cpu-baseline --sustain-s 0 > "$out/bench_under_rocprof.log" 2>&1 || { echo "rocprof bench failed"; exit 1; }
find "$out/prof" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU|SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VALU_FLOPS_FP64" \
    bash tools/pmc.sh "$tag/pmc" --no-extra > "$out/pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "$out/pmc.log"; exit 1; }
PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum" \
    bash tools/pmc.sh "$tag/pmc_batch" --workload batch --no-extra > "$out/pmc_batch.log" 2>&1 || { echo "batch pmc failed"; tail -5 "$out/pmc_batch.log"; exit 1; }
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/cal/p$i" -o run -- \
      python3 tools/pmc_calib.py > "$out/cal_p$i.log" 2>&1 || { echo "calib pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py "$out/cal" > "$out/cal_summary.json"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$out/hostpath" -o run -- \
    python3 tools/host_path_trace.py > "$out/host_path_trace.log" 2>&1 || { echo "host path trace failed"; exit 1; }
python3 tools/host_path_trace.py --summarize "$out/hostpath" > "$out/host_path_summary.json"
cat "$out/bench.json"
