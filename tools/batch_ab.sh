#!/bin/bash
# Batch (C4) A/B on one GPU: for every plot count in $PLOTS (default "128 1024") run the
# batch bench under the default library and each variant, alternating, twice.
# A variant is NAME=VALUE (the default library under that environment) or a name of
# tools/abv/libficp_<name>.so (tools/build_variant.sh).
# usage: PLOTS="128 256" tools/batch_ab.sh FICP_BATCH_STREAMS=1 myvariant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/batch_ab
mkdir -p "$out"
for rep in 1 2; do
  for p in ${PLOTS:-128 1024}; do
    for v in default "$@"; do
      unset FICP_LIB
      envs=""
      case "$v" in
        default) ;;
        *=*) envs="$v" ;;
        *) export FICP_LIB=$PWD/tools/abv/libficp_$v.so ;;
      esac
      log="$out/b${p}_${v//[^A-Za-z0-9_]/_}.log"
      env $envs timeout -k 10 200 python bench.py --workload batch --plots "$p" --steps ${STEPS:-10} \
          --warmup 2 --no-cpu-baseline > "$log" 2>&1 || { echo "batch $p $v failed"; tail -5 "$log"; exit 1; }
      python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
k=d['kernel_ms']; f=lambda n: round(k.get(n,{}).get('ms',0)/max(k.get(n,{}).get('count',1),1)*1e3,1)
print('plots $p $v', round(d['value']), 'plot-it/s', round(d['ms_per_step'],3), 'ms  nn', f('nn_grid_batch'), 'us  sel', f('batch_select'), 'us')"
    done
  done
done
