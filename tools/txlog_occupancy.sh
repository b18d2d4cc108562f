#!/bin/bash
# k_txlog_wave launch time vs launch size: one group per call (MH_TXLOG_CHUNKS=1)
# of N records x 16 entries (R = 8 records per wave: N / 8 waves), from the
# per-kernel HIP events of bench_workloads.py --workload txlog.  Time growing
# per 1024 waves means one resident wave per SIMD; per 2048, two.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/occ
mkdir -p $O
for n in 4096 8192 12288 16384 24576 32768 49152 65536; do
  MH_TXLOG_CHUNKS=1 timeout -k 10 200 python bench_workloads.py --workload txlog --txs $n --steps 20 --warmup 3 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('records %6d waves %5d  k_txlog_wave %.4f ms  call %.3f ms' % ($n, $n//8, d['kernel_ms']['txlog_wave'], d['ms_per_step']))
" | tee -a $O/occ.txt
done
