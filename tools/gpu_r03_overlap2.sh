#!/bin/bash
# Round 3: tx-log validation with the first group checked before the copy
# helper is joined; the fused wire verify's chunk size swept.
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tx.py > $O/t4.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python bench_workloads.py --workload txlog --steps 20 > $O/txlog_$r.json 2> $O/txlog.err
done
for mib in 16 32 64 128; do
  MH_PB_CHUNK_MIB=$mib timeout -k 10 300 python bench_workloads.py --workload wire --steps 5 > $O/wire_$mib.json 2> $O/wire.err
done
