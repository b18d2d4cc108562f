#!/bin/bash
# tx-layer GPU tests incl. the chunked-log mutants, then the device tx-log fuzzer
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tx.py tests/test_gpu_commit.py > $O/pytest_tx.log 2>&1
