#!/bin/bash
# Node-hash K+W row loads ahead of the first block (default build) vs sunk into
# the second block (build_ab/late.so, -DMH_NODE_ROW_LATE), and k_reduce instead
# of k_reduce4 for the wide levels above the leaf kernel (MH_REDUCE4=0):
# htree / tx parity with the default build first, then an interleaved
# single-build / headline A/B.  -> profiles/ab_row_early_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_fullsize.py > $O/pytest_rowearly.log 2>&1
: > $O/rowearly_ab.txt
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline > $O/re.json 2>/dev/null
  echo "$n $(python3 -c "import json;d=json.loads(open('$O/re.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['single_build']['ms_per_build'],d['roofline']['reduce_ms_per_build'])")" >> $O/rowearly_ab.txt
}
for r in 1 2 3; do
  run early MH_DUMMY=1
  run early_r1 MH_REDUCE4=0
  run late MH_LIB_PATH=$PWD/build_ab/late.so
done
cat $O/rowearly_ab.txt
