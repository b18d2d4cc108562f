#!/bin/bash
# k_txlog_group with 256 entry slots per workgroup (one per thread, twice the
# workgroups; default) vs 512 (two per thread, MH_TXLOG_SLOTS=512): tx-log
# parity, then interleaved txlog_timeline / bench runs.
# -> profiles/ab_txlog_slots_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tx.py tests/test_gpu_c_client.py > $O/pytest_txslots.log 2>&1
: > $O/txslots_ab.txt
for r in 1 2 3; do
  for v in 256 512; do
    MH_TXLOG_SLOTS=$v timeout -k 10 120 python tools/txlog_timeline.py > $O/tls.txt 2>&1
    echo "slots=$v timeline $(tail -1 $O/tls.txt)" >> $O/txslots_ab.txt
    MH_TXLOG_SLOTS=$v timeout -k 10 200 python bench_workloads.py --workload txlog --steps 200 > $O/tsb.json 2>/dev/null
    echo "slots=$v bench $(python3 -c "import json;d=json.loads(open('$O/tsb.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['kernel_ms']['txlog_group'])")" >> $O/txslots_ab.txt
  done
done
cat $O/txslots_ab.txt
