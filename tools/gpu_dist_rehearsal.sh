#!/bin/bash
# Two ranks sharing the one GPU of a test box over gloo (MH_DIST_BACKEND=gloo):
# rehearses bench.py's multi-rank path (clock pre-warm decisions, root
# all-gather, max-over-ranks timing) without RCCL's one-rank-per-GPU rule.
# No scaling is claimed from it: both ranks share one device.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MH_DIST_BACKEND=gloo HIP_VISIBLE_DEVICES=0 timeout -k 10 300 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dist2.json 2> gpurun_out/dist2.err
rc=$?
cat gpurun_out/dist2.json; grep -v amdgpu.ids gpurun_out/dist2.err | tail -5
exit $rc
