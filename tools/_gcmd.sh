mkdir -p gpurun_out
for mode in 0 1 2 3 4; do for os in "" onesweep; do FICP_SORT=$os timeout -k 10 60 ./tools/sortcheck 1000000 3 1 $mode 1 > gpurun_out/sc.log 2>&1; echo "mode $mode $os rc=$? $(tail -n 1 gpurun_out/sc.log)"; done; done
timeout -k 10 60 ./tools/sortcheck 1000 3 1 0 1 > gpurun_out/sc.log 2>&1; echo "small rc=$? $(tail -n 1 gpurun_out/sc.log)"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "rcp=$?"; tail -n 3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench.log 2>&1; echo "rc=$?"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
bash tools/profile.sh prof_c3 --steps 10 > /dev/null 2>&1; echo "prof c3 rc=$?"
