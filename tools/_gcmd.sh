mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "rcp=$?"; tail -n 3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --workload c5 --c5-size 2000000 --local-shards 4 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1; echo "c5 rc=$?"; tail -c 700 gpurun_out/bench_c5.log
