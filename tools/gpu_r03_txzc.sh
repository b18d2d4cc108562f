#!/bin/bash
# a14 with the last chunk of a pinned log fetched by its group's kernel over
# PCIe (default) vs DMA'd like the others (MH_TXLOG_ZC=0): tx-log parity, then
# the interleaved bench A/B and plain txlog_timeline runs of both.
# -> profiles/ab_txlog_zc_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
V1=zc E1=MH_DUMMY=1 V2=dma E2=MH_TXLOG_ZC=0 V3=chain E3=MH_TXLOG_FUSED=0 ROUNDS=4 bash tools/gpu_r03_txfused.sh
for r in 1 2 3; do
  MH_TXLOG_TRACE=1 timeout -k 10 120 python tools/txlog_timeline.py > $O/tl_zc_plain$r.txt 2>&1
  MH_TXLOG_ZC=0 MH_TXLOG_TRACE=1 timeout -k 10 120 python tools/txlog_timeline.py > $O/tl_dma_plain$r.txt 2>&1
done
