#!/bin/bash
# A/B: tx-log chunks on the copy stream (default) vs on the compute stream
# (MH_TXLOG_COPY_ON_COMPUTE=1), interleaved; txlog tests under the knob first.
set -eo pipefail
O=gpurun_out
mkdir -p $O
MH_TXLOG_COPY_ON_COMPUTE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tx.py -k txlog > $O/pytest_txswap.log 2>&1
: > $O/txswap_ab.txt
for r in 1 2 3; do
  echo "base $(timeout -k 10 120 python tools/txlog_timeline.py 2>/dev/null | tail -1)" >> $O/txswap_ab.txt
  echo "swap $(MH_TXLOG_COPY_ON_COMPUTE=1 timeout -k 10 120 python tools/txlog_timeline.py 2>/dev/null | tail -1)" >> $O/txswap_ab.txt
done
cat $O/txswap_ab.txt
