cd $GRAFT_REPO_ROOT
out=gpurun_out/r4b; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 bash tools/wincheck.sh > $out/wincheck.txt 2>&1; echo "wincheck rc=$?"; grep -E "summary|MISMATCH" $out/wincheck.txt | head -30
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_window.py \
   tests/test_gpu_configs.py tests/test_gpu_batch.py -k "window or c3 or batch_vs_oracle or far_apart or golden_runs" > $out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -3 $out/pytest.log
[ $rc -ne 0 ] && exit 1
BENCH_ARGS="--no-extra --steps 40" timeout -k 10 800 bash tools/ab_bench.sh FICP_WIN_NN=0 nopass
PLOTS="256 512" STEPS=6 timeout -k 10 500 bash tools/batch_ab.sh FICP_BATCH_QPT_MIN=1 FICP_BATCH_QPT=0
