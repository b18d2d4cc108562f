#!/bin/bash
# C5 htree proof re-hash with the next term's load issued before each step's
# node hash (default) vs loaded at the top of the step (build_ab/noprefetch.so,
# -DMH_C5_NO_PREFETCH): verify parity first, then an interleaved c5 A/B.
# -> profiles/ab_c5_prefetch_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "verify or c5 or proof" > $O/pytest_c5pf.log 2>&1
: > $O/c5pf_ab.txt
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench_workloads.py --workload c5 --no-ahtree > $O/c5.json 2>/dev/null
  echo "$n $(python3 -c "import json;d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print(d['value'],d.get('ms_per_step'),d.get('kernel_ms'))")" >> $O/c5pf_ab.txt
}
for r in 1 2 3; do
  run prefetch MH_DUMMY=1
  run noprefetch MH_LIB_PATH=$PWD/build_ab/noprefetch.so
done
cat $O/c5pf_ab.txt
