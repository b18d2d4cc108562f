#!/bin/bash
# Rotating A/B of the headline bench over environment settings on one box:
# VARIANTS="A=1 B=2 ..." style, each a space-free "NAME=VALUE[,NAME=VALUE]" or "base".
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    envs=""
    [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-2000} ${BENCH_ARGS} > gpurun_out/abe.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/abe.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['sha']['frac'], d['single_build']['ms_per_build'])"
  done
done
