#!/bin/bash
# Round 3: wire verify chunk sweep with the zero-copy total read-back; a
# kernel + memory-copy trace of the tx-log validation.
set -eo pipefail
O=gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pb_decode.py > $O/t5.log 2>&1
for mib in 16 32 64 128; do
  MH_PB_CHUNK_MIB=$mib timeout -k 10 300 python bench_workloads.py --workload wire --steps 5 > $O/wire_$mib.json 2> $O/wire.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof_txlog -o txlog -- python bench_workloads.py --workload txlog --steps 3 --warmup 1 > $O/txlog_prof.json 2> $O/txlog_prof.err
