#!/bin/bash
# Full GPU suite, then interleaved A/Bs (headline + ragged) of the in-tree
# library vs build/ab/$AB_LIB on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/ab_suite.log 2>&1; rc=$?
tail -4 gpurun_out/ab_suite.log
[ $rc -ne 0 ] && exit $rc
STEPS=${HSTEPS:-1000} bash tools/ab_lib.sh || exit 1
for i in 1 2 3; do
  for v in base alt; do
    if [ $v = alt ]; then export MH_LIB_PATH=build/ab/$AB_LIB; else unset MH_LIB_PATH; fi
    timeout -k 10 200 python bench_workloads.py --workload ragged --steps 20 --no-check > gpurun_out/abr_$v.json 2> gpurun_out/abr_$v.err || { tail -5 gpurun_out/abr_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abr_$v.json')); print('ragged $v', d['value'], d['ms_per_step'], d['kernel_ms'], d['sha']['frac'])"
  done
done
