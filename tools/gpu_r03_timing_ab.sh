#!/bin/bash
# A/B of the headline: per-kernel timing events off in the timed region
# (default) vs on (--timing-in-region), interleaved, the driver's 20-step
# command and the default 2000 steps; then the tx-log copy-stream A/B.
set -eo pipefail
O=gpurun_out
mkdir -p $O
: > $O/timing_ab.txt
for r in 1 2 3; do
  for v in off on; do
    extra=""; [ $v = on ] && extra="--timing-in-region"
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $extra > $O/tab.json 2>/dev/null
    echo "$v steps20 $(python3 -c "import json;d=json.loads(open('$O/tab.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['contended_kernel_ms'])")" >> $O/timing_ab.txt
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2000 $extra > $O/tab.json 2>/dev/null
    echo "$v steps2000 $(python3 -c "import json;d=json.loads(open('$O/tab.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['contended_kernel_ms'])")" >> $O/timing_ab.txt
  done
done
cat $O/timing_ab.txt
bash tools/gpu_r03_txswap.sh
