#!/bin/bash
# Round-3 iteration 7: parity after the run-start/loop-init merge, C3 rate, a C3 kernel
# timeline (every kernel of one run), and the NN counter passes: traffic,
# TA/TD busy, lane utilisation, wait cycles; plus the 8-B-per-lane FETCH/WRITE calibration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it7
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_ties_golden.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --steps 40 --warmup 5 > "$out/c3_$rep.log" 2>&1 || { echo "c3 bench failed"; tail -5 "$out/c3_$rep.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/c3_$rep.log').read().strip().splitlines()[-1]); print('c3', round(d['value']), round(d['ms_per_step'],3), d['roofline']['achieved'], d.get('iteration_roofline',{}).get('frac'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
    python3 bench.py --no-extra --no-cpu-baseline --steps 4 --warmup 1 > "$out/prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/timeline.py "$out/prof/run_kernel_trace.csv" k_run_start -v > "$out/timeline.txt" 2>&1
tail -22 "$out/timeline.txt"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VALU_FLOPS_FP64"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/pmc/p$i" -o run -- \
      python3 bench.py --no-extra --no-cpu-baseline --steps 2 --warmup 1 > "$out/pmc_p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$out/pmc_p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$out/pmc" > "$out/pmc_summary.json"
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/cal/p$i" -o run -- \
      python3 tools/pmc_calib.py > "$out/cal_p$i.log" 2>&1 || { echo "calib pass $i failed"; tail -5 "$out/cal_p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$out/cal" > "$out/cal_summary.json"
python3 -c "
import json
d = json.load(open('$out/pmc_summary.json'))
for k, v in d.items():
    if 'nn_grid' in k: print(k, {a: (round(b, 1) if isinstance(b, float) else b) for a, b in v.items()})
c = json.load(open('$out/cal_summary.json'))
for k, v in c.items():
    if 'apply' in k: print('calib', k, v.get('fetch_bytes_raw'), v.get('write_bytes'), 'known', 16 * (1 << 24))
"
