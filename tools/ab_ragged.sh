#!/bin/bash
# Ragged-entry parity, then an interleaved A/B of the ragged workload: in-tree
# library (base) vs build/ab/$AB_LIB (alt), one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_c_client.py \
  tests/test_gpu_fullsize.py::test_ragged_full_size_vs_oracle \
  > gpurun_out/ab_ragged_tests.log 2>&1; rc=$?
tail -5 gpurun_out/ab_ragged_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in base alt; do
    if [ $v = alt ]; then export MH_LIB_PATH=build/ab/$AB_LIB; else unset MH_LIB_PATH; fi
    timeout -k 10 200 python bench_workloads.py --workload ragged --steps ${STEPS:-20} ${RAGGED_ARGS} > gpurun_out/abr_$v.json 2> gpurun_out/abr_$v.err || { tail -5 gpurun_out/abr_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abr_$v.json')); print('$v', d['value'], d['ms_per_step'], d['kernel_ms'], d['sha']['frac'], d['oracle_match'])"
  done
done
