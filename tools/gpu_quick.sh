#!/bin/bash
# quick loop: GPU parity suite (fast files), ragged + headline benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_commit.py tests/test_gpu_tx.py tests/test_gpu_c_client.py \
  tests/test_gpu_fullsize.py::test_ragged_full_size_vs_oracle ${EXTRA_TESTS} \
  > gpurun_out/quick_tests.log 2>&1; rc=$?
tail -5 gpurun_out/quick_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_workloads.py --workload ragged --steps 10 > gpurun_out/w_ragged.json 2> gpurun_out/w_ragged.err || { tail -5 gpurun_out/w_ragged.err; exit 1; }
cat gpurun_out/w_ragged.json
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
