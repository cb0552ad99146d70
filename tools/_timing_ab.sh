cd $GRAFT_REPO_ROOT
for m in none first all; do timeout -k 10 200 python bench.py --no-cpu-baseline --nn-timing $m > gpurun_out/t_$m.log 2>&1 || exit 1; python3 -c "
import json,sys; d=json.loads(open('gpurun_out/t_$m.log').read().strip().splitlines()[-1]); print('$m', round(d['value'],1), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],2), d['roofline']['launches'])"; done
