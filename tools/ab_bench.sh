#!/bin/bash
# Bench the default library against variants (tools/abv/libficp_<name>.so), alternating
# runs; prints it/s and NN launch time.  usage: tools/ab_bench.sh name1 [name2 ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in default "$@"; do
    unset FICP_LIB
    envs=""
    case "$v" in
      default) ;;
      *=*) envs="$v" ;;  # NAME=VALUE: the default library under that environment
      *) export FICP_LIB=$PWD/tools/abv/libficp_$v.so ;;
    esac
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --sustain-s 0 ${BENCH_ARGS} > "gpurun_out/ab/$v.log" 2>&1 || { echo "$v failed"; tail -5 "gpurun_out/ab/$v.log"; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab/$v.log').read().strip().splitlines()[-1])
print('$v', round(d['value'],1), 'it/s', round(d['ms_per_step'],4), 'ms/step  nn', round(d['roofline']['avg_launch_us'],2), 'us', d.get('selection_paths', ''))"
  done
done
