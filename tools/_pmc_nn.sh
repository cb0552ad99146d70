cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmcnn
mkdir -p $out
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VALU_FLOPS_FP64 SQ_LEVEL_WAVES TA_TA_BUSY_sum TA_BUSY_max" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TD_TD_BUSY_sum TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $out > $out/summary.json
python3 -c "
import json; d=json.load(open('$out/summary.json'))
for k,v in d.items():
    if 'nn_grid' in k or 'sel_' in k or 'fit' in k: print(k, {a:round(b,1) for a,b in v.items()})"
