#!/bin/bash
# Round-3 iteration 22: batch shares with the fused fit pass loading 8 / 10 / 16 rows per
# thread per round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/it22
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # plots, label, lib
  local p=$1 lab=$2 lib=$3
  FICP_LIB=$lib timeout -k 10 150 python bench.py --workload batch --plots $p --steps 10 --warmup 2 --no-cpu-baseline > "$out/b${p}_$lab.log" 2>&1 || { echo "batch $p $lab failed"; tail -5 "$out/b${p}_$lab.log"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/b${p}_$lab.log').read().strip().splitlines()[-1]); print('plots $p $lab', round(d['value']), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  for p in 128 1024; do
    run $p fu8 $PWD/coregistrationgame_amd/libficp.so || exit 1
    run $p fu10 $PWD/tools/ab/libficp_bfu10.so || exit 1
    run $p fu16 $PWD/tools/ab/libficp_bfu16.so || exit 1
  done
done
