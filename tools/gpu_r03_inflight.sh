#!/bin/bash
# builds in flight A/B (bench.py --inflight), interleaved, 2000 steps
set -eo pipefail
O=gpurun_out
mkdir -p $O
: > $O/inflight_ab.txt
for r in 1 2; do
  for d in 3 4 2 6; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --inflight $d > $O/inf.json 2>/dev/null
    echo "inflight $d $(python3 -c "import json;d=json.loads(open('$O/inf.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" >> $O/inflight_ab.txt
    timeout -k 10 200 python bench.py --no-cpu-baseline --inflight $d --steps 20 --warmup 5 > $O/inf.json 2>/dev/null
    echo "inflight $d steps20 $(python3 -c "import json;d=json.loads(open('$O/inf.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" >> $O/inflight_ab.txt
  done
done
cat $O/inflight_ab.txt
