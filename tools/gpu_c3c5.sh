#!/bin/bash
# Parity of the ahtree / verify kernels, then C3 and C5 with and without the
# LDS node-schedule table (MH_NODE_TABLE=0 restores the plain node hash in the
# ahtree append path; the verify kernels always use the table).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_c3c5.log 2>&1 || { tail -30 gpurun_out/pytest_c3c5.log; exit 1; }
tail -3 gpurun_out/pytest_c3c5.log
for r in 1 2; do
  for cfg in ${C3_CONFIGS:-MH_NODE_TABLE=0 MH_SPINE_PREFETCH=0 MH_SPINE_PREFETCH=1}; do
    env $(echo "$cfg" | tr ',' ' ') timeout -k 10 180 python bench_workloads.py --workload c3 --steps 5 > gpurun_out/c3.json || exit 1
    echo "$cfg $(cat gpurun_out/c3.json)"
  done
done
timeout -k 10 180 python bench_workloads.py --workload c5 --steps 5 > gpurun_out/c5.json || exit 1
cat gpurun_out/c5.json
