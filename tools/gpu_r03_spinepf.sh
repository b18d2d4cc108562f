#!/bin/bash
# C3 ahtree batch append: the spine's next left node loaded under the current
# step's node hash (pf6: -DMH_SPINE_PREFETCH at the 80-VGPR cap, 6 spilled;
# pf4: the same with 4 waves per SIMD, no spill) vs the shipped kernel (base):
# append parity with each build, then an interleaved c3 A/B.
# -> profiles/ab_spine_prefetch_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
for v in pf6 pf4; do
  MH_LIB_PATH=$PWD/build_ab/$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_formats.py -k "ahtree or append or c3" > $O/pytest_spine_$v.log 2>&1
done
: > $O/spine_ab.txt
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench_workloads.py --workload c3 > $O/c3.json 2>/dev/null
  echo "$n $(python3 -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]);print(d['value'],d.get('ms_per_step'),d.get('kernel_ms'))")" >> $O/spine_ab.txt
}
for r in 1 2 3; do
  run base MH_DUMMY=1
  run pf6 MH_LIB_PATH=$PWD/build_ab/pf6.so
  run pf4 MH_LIB_PATH=$PWD/build_ab/pf4.so
done
cat $O/spine_ab.txt
