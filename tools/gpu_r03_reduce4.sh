#!/bin/bash
# A/B: first reduce launch with two in-lane levels (k_reduce4, default) vs one
# node per lane (MH_REDUCE4=0), interleaved: headline + single build
set -eo pipefail
O=gpurun_out
mkdir -p $O
MH_REDUCE4=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "htree or build" > $O/pytest_r4.log 2>&1
: > $O/reduce4_ab.txt
for r in 1 2 3; do
  for v in 1 0; do
    MH_REDUCE4=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/r4.json 2>/dev/null
    echo "reduce4=$v $(python3 -c "import json;d=json.loads(open('$O/r4.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['single_build']['ms_per_build'],d['roofline']['reduce_ms_per_build'])")" >> $O/reduce4_ab.txt
  done
done
cat $O/reduce4_ab.txt
