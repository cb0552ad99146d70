#!/bin/bash
# Round-3 first measurements: host-path breakdown, batch shares (1024/512/256/128 plots on
# one GPU = the per-rank shares of N = 1/2/4/8), NN PMC passes.  usage: tools/r3_probe.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/r3probe
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/host_probe.py > "$out/host.json" 2> "$out/host.err" || { echo "host probe failed"; tail -5 "$out/host.err"; exit 1; }
cat "$out/host.json"
for p in 1024 512 256 128; do
    timeout -k 10 240 python3 bench.py --workload batch --plots $p --no-cpu-baseline --steps 10 --warmup 2 > "$out/batch_$p.log" 2>&1 || { echo "batch $p failed"; tail -5 "$out/batch_$p.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$out/batch_$p.log').read().strip().splitlines()[-1]); print($p, round(d['value']), round(d['ms_per_step'],3), {k:round(v['ms'],3) for k,v in d['kernel_ms'].items()})"
done
