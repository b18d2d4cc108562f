#!/bin/bash
# A/B of library builds / env configs / bench args, alternated ROUNDS times.
# AB_CONFIGS: space-separated entries "ENV1=a,ENV2=b;--bench-arg value"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
for cfg in ${AB_CONFIGS}; do
  envs="${cfg%%;*}"; args=""
  [[ "$cfg" == *";"* ]] && args="${cfg#*;}"
  envs=$(echo "$envs" | tr ',' ' '); args=$(echo "$args" | tr '_' ' ')
  env $envs timeout -k 10 120 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline $args > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$cfg', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step kernel', r['kernel_ms'], 'reduce', r['reduce_ms_per_step'], 'sha', r['sha']['frac'], 'iso_ms', r.get('isolated_kernel_ms'))"
done
done
