#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_debug.py > gpurun_out/debug.log 2>&1; rc=$?
cat gpurun_out/debug.log | grep -v amdgpu.ids
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:randomly > gpurun_out/pytest_gpu.log 2>&1
tail -40 gpurun_out/pytest_gpu.log
