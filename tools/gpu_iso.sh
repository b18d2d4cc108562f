#!/bin/bash
# Isolated leaf-kernel duration vs in-kernel workgroup-subtree depth (and any
# other env configs in ISO_CONFIGS), plus the hardware-id probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -x tools/hwid_probe ]; then
  timeout -k 10 60 tools/hwid_probe > gpurun_out/hwid.txt || exit 1
fi
for cfg in ${ISO_CONFIGS:-MH_WG_LEVELS=0 MH_WG_LEVELS=4 MH_WG_LEVELS=8}; do
  envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 3 --inflight 2 --no-cpu-baseline > gpurun_out/iso.json 2>gpurun_out/iso.err || { tail -5 gpurun_out/iso.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/iso.json'));r=d['roofline'];print('$cfg', d['value'], 'GiB/s iso_kernel_ms', r['isolated_kernel_ms'], 'sha', r['isolated_sha_frac'])"
done
