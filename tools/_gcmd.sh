mkdir -p gpurun_out
for mode in 0 2; do timeout -k 10 60 ./tools/sortcheck 1000000 3 1 $mode 1 > gpurun_out/sc_$mode.log 2>&1; echo "mode $mode rc=$? $(tail -n 1 gpurun_out/sc_$mode.log)"; done
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "rcp=$?"; tail -n 3 gpurun_out/pytest_gpu.log
bash tools/profile.sh prof_c3 --steps 10 > /dev/null 2>&1; echo "prof c3 rc=$?"
bash tools/profile.sh prof_batch --workload batch --steps 3 --warmup 1 > /dev/null 2>&1; echo "prof batch rc=$?"
grep '^{' gpurun_out/prof_c3/bench.log | cut -c1-400
grep '^{' gpurun_out/prof_batch/bench.log | cut -c1-400
