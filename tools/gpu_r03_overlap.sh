#!/bin/bash
# Round 3: the PCIe / compute overlap of the fused DualProofV2 wire verify and
# the tx-log validation (parity first, then the two bench lines).
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tx.py tests/test_gpu_pb_decode.py > $O/t3.log 2>&1
timeout -k 10 300 python bench_workloads.py --workload txlog --steps 20 > $O/txlog.json 2> $O/txlog.err
timeout -k 10 300 python bench_workloads.py --workload wire --steps 5 > $O/wire.json 2> $O/wire.err
