#!/bin/bash
# top-of-tree node hashes with the schedule on a second wave (default) vs not
# (MH_SPLIT_TOP=0): htree parity first, then an interleaved single-build /
# headline A/B
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py -k "htree or build or shard or c2" > $O/pytest_split.log 2>&1
: > $O/split_ab.txt
for r in 1 2 3; do
  for v in 1 0; do
    MH_SPLIT_TOP=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/sp.json 2>/dev/null
    echo "split=$v $(python3 -c "import json;d=json.loads(open('$O/sp.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['single_build']['ms_per_build'],d['roofline']['reduce_ms_per_build'])")" >> $O/split_ab.txt
  done
done
cat $O/split_ab.txt
