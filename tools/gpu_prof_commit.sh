#!/bin/bash
# Kernel + memory-copy trace of the commit workload (no counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/profc" -o run -- python3 "$GRAFT_REPO_ROOT/bench_workloads.py" --workload commit --steps 2 --warmup 1 ${COMMIT_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/profc.log" 2>&1; rc=$?
tail -3 "$GRAFT_REPO_ROOT/gpurun_out/profc.log"
find "$GRAFT_REPO_ROOT/gpurun_out/profc" -name "*.csv"
exit $rc
