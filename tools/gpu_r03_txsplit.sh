#!/bin/bash
# a14 two-phase hop: the tx GPU tests, then the txlog workload with the
# phase trace (3 runs) for the <= 1.6 ms target.
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tx.py > $O/pytest_tx.log 2>&1
for r in 1 2 3; do
  MH_TXLOG_TRACE=1 timeout -k 10 200 python bench_workloads.py --workload txlog --steps 20 > $O/txlog_$r.json 2> $O/txlog_$r.err
done
