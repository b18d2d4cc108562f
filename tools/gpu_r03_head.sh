#!/bin/bash
# Every -m gpu test and smoke() at HEAD (the driver's round-end checks).
set -eo pipefail
O=gpurun_out/head
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 600 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
