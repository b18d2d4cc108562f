#!/bin/bash
# Ragged-entry path on the GPU: parity tests, then the ragged workload with the
# length-class sort and without it (MH_VARLEN_NOSORT=1), one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_commit.py tests/test_gpu_tx.py tests/test_gpu_c_client.py \
  tests/test_gpu_fullsize.py::test_ragged_full_size_vs_oracle \
  > gpurun_out/ragged_tests.log 2>&1; rc=$?
tail -15 gpurun_out/ragged_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_workloads.py --workload ragged --steps 10 > gpurun_out/w_ragged.json 2> gpurun_out/w_ragged.err || { tail -5 gpurun_out/w_ragged.err; exit 1; }
cat gpurun_out/w_ragged.json
MH_VARLEN_NOSORT=1 timeout -k 10 300 python bench_workloads.py --workload ragged --steps 10 --no-check > gpurun_out/w_ragged_nosort.json 2> gpurun_out/w_ragged_nosort.err || { tail -5 gpurun_out/w_ragged_nosort.err; exit 1; }
cat gpurun_out/w_ragged_nosort.json
timeout -k 10 300 python bench_workloads.py --workload commit > gpurun_out/w_commit.json 2> gpurun_out/w_commit.err || { tail -5 gpurun_out/w_commit.err; exit 1; }
cat gpurun_out/w_commit.json
