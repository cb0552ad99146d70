#!/bin/bash
# Round-3 iteration: new tests, fused-fit A/B at C3, batch-select phase profile and a
# kernel timeline of the 128-plot batch share.  Stops at the first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it2
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_errors.py tests/test_ties_golden.py "tests/test_gpu_batch.py::test_source_mode_pack_overflow_is_exact" \
    "tests/test_gpu_parity.py" > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 400 bash tools/ab_bench.sh FICP_FUSE_FIT=1 || exit 1
FICP_LIB=$PWD/tools/ab/libficp_bselprof.so timeout -k 10 120 python bench.py --workload batch --plots 128 --steps 2 --warmup 1 --no-cpu-baseline > "$out/bselprof.log" 2>&1 || { echo "bselprof failed"; tail -5 "$out/bselprof.log"; exit 1; }
grep BSEL "$out/bselprof.log" | head -12
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof128" -o run -- \
    python3 bench.py --workload batch --plots 128 --steps 3 --warmup 1 --no-cpu-baseline > "$out/prof128.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/timeline.py "$out/prof128/run_kernel_trace.csv" k_batch_init > "$out/timeline128.txt" 2>&1
head -30 "$out/timeline128.txt"
