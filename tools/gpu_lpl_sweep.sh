#!/bin/bash
# Sweep lanes-per-leaf-group (MH_LPL) x workgroup subtree levels (MH_WG_LEVELS)
# on C2: headline (3 in flight), isolated leaf launch and single-build time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/lpl_sweep.txt
: > $out
for pass in 1 2; do
  for cfg in ${CFGS:-4_2 2_2 2_3 4_0 2_1 1_2}; do
    set -- ${cfg/_/ }
    MH_LPL=$1 MH_WG_LEVELS=$2 timeout -k 10 120 python bench.py --steps 1000 --no-cpu-baseline > gpurun_out/s.json 2>/dev/null || exit 1
    python -c "
import json;d=json.load(open('gpurun_out/s.json'));r=d['roofline']
print('pass $pass lpl $1 wgl $2', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['sha']['frac'], r['reduce_ms_per_build'], d['single_build']['ms_per_build'])" | tee -a $out
  done
done
