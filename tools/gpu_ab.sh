#!/bin/bash
# A/B: parity subset + bench under several env settings (one process each).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for cfg in ${AB_CONFIGS}; do
  env $(echo $cfg | tr ',' ' ') timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$cfg', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step kernel', r['kernel_ms'], 'reduce', r['reduce_ms_per_step'], 'valu', r['valu']['frac'])"
done
