#!/bin/bash
# interleaved A/B of the tx-log validation: build/ab/libold.so vs the in-tree library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export MH_LIB_PATH=build/ab/libold.so; else unset MH_LIB_PATH; fi
    timeout -k 10 300 python bench_workloads.py --workload txlog --steps ${STEPS:-20} > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['ms_per_step'], d['host_hop_only_ms'], d['h2d_only_ms'], d['pageable_input']['ms_per_step'], d['kernel_ms'])"
  done
done
