#!/bin/bash
# Round 3 validation: every -m gpu test, smoke(), the driver's bench command and
# a rocprofv3 kernel-trace/stats run of the same command.
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 1500 python -u -m pytest -m gpu -v --timeout 900 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
