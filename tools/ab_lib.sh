#!/bin/bash
# interleaved A/B of the headline bench: in-tree library vs build/ab/$AB_LIB
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base alt; do
    if [ $v = alt ]; then export MH_LIB_PATH=build/ab/$AB_LIB; else unset MH_LIB_PATH; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-1000} ${BENCH_ARGS} > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['sha']['frac'], d['single_build']['ms_per_build'])"
  done
done
