mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "rcp=$?"; tail -n 30 gpurun_out/pytest_gpu.log
