mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "rcp=$?"; tail -n 2 gpurun_out/pytest_gpu.log
run() { FICP_LIB=$1 FICP_GRID_PER_CELL=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_dbg.log 2>&1; echo "lib=$1 pc=$2 rc=$?"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_dbg.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['iterations_per_step'])"; }
run "" 2.0; run "" 1.0; for u in 1 2 8; do run coregistrationgame_amd/dev/libficp_u$u.so 1.0; done
