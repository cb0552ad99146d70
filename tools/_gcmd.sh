mkdir -p gpurun_out
PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" bash tools/pmc.sh pmc_c3 > /dev/null 2>&1; echo rc=$?
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_c3/summary.json'))
for x in d:
  if x.startswith('k_nn_grid') or x.startswith('k_os'): print(x, {a:round(b,1) for a,b in d[x].items()})"
