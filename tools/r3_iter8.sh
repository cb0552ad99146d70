#!/bin/bash
# Round-3 iteration 8: parity (keys from r, pooled host arrays, two sub-batches from 64
# plots), C3 A/B of stored vs derived keys, the selection phase profile (SEL_PROF build),
# then the default bench line (host path with pooled pinned layers, app scale, shares).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it8
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_gpu_batch.py tests/test_ties_golden.py \
    > "$out/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
BENCH_ARGS="--no-extra --steps 40 --warmup 5" timeout -k 10 400 bash tools/ab_bench.sh FICP_NN_KEYS=1 || exit 1
FICP_LIB=$PWD/tools/ab/libficp_selprof.so timeout -k 10 120 python bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 1 > "$out/selprof.log" 2>&1 || { echo "selprof failed"; tail -5 "$out/selprof.log"; exit 1; }
grep SELPROF "$out/selprof.log" | head -14
timeout -k 10 600 python bench.py > "$out/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$out/bench.log"; exit 1; }
python3 - "$out/bench.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 4), "nn_us", d["roofline"]["avg_launch_us"], "frac", round(d["roofline"]["frac"], 3))
print("iteration_roofline", d.get("iteration_roofline"))
print("host_path", json.dumps(d.get("host_path"))[:900])
print("app_scale", d.get("app_scale_join"))
print("shares", json.dumps(d.get("batch_shares"))[:600])
PY
