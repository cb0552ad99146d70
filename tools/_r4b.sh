cd $GRAFT_REPO_ROOT
out=gpurun_out/r4b; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 bash tools/wincheck.sh > $out/wincheck.txt 2>&1; echo "wincheck rc=$?"; grep -E "summary|MISMATCH" $out/wincheck.txt | head -30
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_window.py \
   tests/test_gpu_configs.py -k "window or c3" > $out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "PASS|FAIL|ERROR|passed|failed" $out/pytest.log | tail -20
[ $rc -ne 0 ] && exit 1
BENCH_ARGS="--no-extra --steps 40" timeout -k 10 600 bash tools/ab_bench.sh FICP_WIN_NN=0
