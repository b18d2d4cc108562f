#!/bin/bash
# innerHash message of metadata-free headers built in registers (default) vs
# assembled byte by byte in a scratch slot (build_ab/base.so): tx parity, then
# interleaved a14 timeline / VerifyDocument runs.
# -> profiles/ab_inner_regs_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tx.py tests/test_gpu_c_client.py tests/test_gpu_pb_decode.py > $O/pytest_innerreg.log 2>&1
: > $O/innerreg_ab.txt
for r in 1 2 3; do
  for v in regs base; do
    E=MH_DUMMY=1; [ $v = base ] && E=MH_LIB_PATH=$PWD/build_ab/base.so
    env $E timeout -k 10 120 python tools/txlog_timeline.py > $O/tli.txt 2>&1
    env $E timeout -k 10 200 python bench_workloads.py --workload document > $O/doc.json 2>/dev/null
    echo "$v a14 $(tail -1 $O/tli.txt) | document $(python3 -c "import json;d=json.loads(open('$O/doc.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" >> $O/innerreg_ab.txt
  done
done
cat $O/innerreg_ab.txt
