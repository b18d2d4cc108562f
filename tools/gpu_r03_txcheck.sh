#!/bin/bash
# tx-layer parity with the shipped a14 path (fused group kernel, DMA'd chunks),
# then a14 through the C ABI alone (tools/txlog_bench, three runs of 200 calls).
# -> profiles/txlog_cabi_r03b.jsonl
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tx.py tests/test_gpu_commit.py > $O/pytest_txcheck.log 2>&1
: > $O/txlog_cabi.jsonl
for r in 1 2 3; do
  LD_LIBRARY_PATH=$PWD/immustore_amd timeout -k 10 120 ./tools/txlog_bench 200 >> $O/txlog_cabi.jsonl
done
cat $O/txlog_cabi.jsonl
