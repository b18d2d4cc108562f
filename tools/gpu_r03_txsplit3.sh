#!/bin/bash
# a14 final: tx + commit GPU tests, the txlog workload 3x (timed pass without
# per-kernel timing events), interleaved chunk-count sweep.
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tx.py tests/test_gpu_commit.py > $O/pytest_tx.log 2>&1
for r in 1 2 3; do
  timeout -k 10 200 python bench_workloads.py --workload txlog --steps 50 > $O/txlog_$r.json 2> $O/txlog_$r.err
done
for r in 1 2; do for ch in 2 3 4 5; do
  MH_TXLOG_CHUNKS=$ch timeout -k 10 200 python bench_workloads.py --workload txlog --steps 50 > $O/txlog_ch${ch}_$r.json 2>/dev/null
done; done
