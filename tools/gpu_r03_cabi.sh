#!/bin/bash
# Round 3: the driver's bench command, the one-process C-ABI mode (mh_multi_*
# with a real RCCL clique of one device), and the leaf kernel's workgroup
# residency (tools/wg_trace) at two and four entries per lane.
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
timeout -k 10 300 python bench.py --api cabi --gpus 1 --steps 200 --no-cpu-baseline > $O/bench_cabi_c2.json 2> $O/bench_cabi_c2.err
timeout -k 10 300 python bench.py --api cabi --gpus 1 --config c4 --steps 10 --no-cpu-baseline > $O/bench_cabi_c4.json 2> $O/bench_cabi_c4.err
timeout -k 10 120 ./tools/wg_trace 600 0 > $O/wgt_lpl2_iso.json
MH_LPL=4 timeout -k 10 120 ./tools/wg_trace 600 0 > $O/wgt_lpl4_iso.json
timeout -k 10 120 ./tools/wg_trace 600 1 > $O/wgt_lpl2_cont.json
python tools/wg_trace_summary.py $O/wgt_lpl2_iso.json $O/wgt_lpl4_iso.json $O/wgt_lpl2_cont.json > $O/wgt_summary.jsonl
