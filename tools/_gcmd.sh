mkdir -p gpurun_out
for mode in 0 1 2 3 4; do
 for orig in 0 1; do
  timeout -k 10 60 ./tools/sortcheck 1000000 3 $orig $mode $orig > gpurun_out/sc_${mode}_${orig}.log 2>&1 || true
  echo "mode=$mode orig=$orig: $(tail -1 gpurun_out/sc_${mode}_${orig}.log) $(head -1 gpurun_out/sc_${mode}_${orig}.log)"
 done
done
FICP_SORT=onesweep timeout -k 10 60 ./tools/sortcheck 1000000 3 0 2 0 > gpurun_out/sc_os_2.log 2>&1; echo "onesweep mode 2: $(tail -1 gpurun_out/sc_os_2.log)"
FICP_CHECK=2 timeout -k 10 300 python tools/debug_bench.py 1000000 3 > gpurun_out/dbg_check2.log 2>&1; echo "rc2=$?" >> gpurun_out/dbg_check2.log
tail -n 3 gpurun_out/dbg_check2.log
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "rcp=$?" >> gpurun_out/pytest_gpu.log
tail -n 5 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; echo "rcb=$?"; tail -c 3000 gpurun_out/bench.log
