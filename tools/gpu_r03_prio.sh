#!/bin/bash
# Round 3 A/B: falling wave priority in k_entries_fixed (MH_SETPRIO=1) vs off,
# interleaved on one box: the driver's command (3 builds in flight, isolated
# launch, single build) and a workgroup trace of an isolated launch each.
set -eo pipefail
O=gpurun_out
mkdir -p $O
: > $O/ab_prio.jsonl
for r in 1 2 3; do
  for p in 0 1; do
    MH_SETPRIO=$p timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline > $O/ab_prio_tmp.json 2>/dev/null
    python -c "import json,sys;d=json.load(open('$O/ab_prio_tmp.json'));print(json.dumps({'prio':$p,'value':d['value'],'ms':d['ms_per_step'],'iso':d['roofline']['kernel_ms'],'single':d['single_build']['ms_per_build']}))" >> $O/ab_prio.jsonl
  done
done
MH_SETPRIO=0 timeout -k 10 120 ./tools/wg_trace 600 0 > $O/wgt_prio0.json
MH_SETPRIO=1 timeout -k 10 120 ./tools/wg_trace 600 0 > $O/wgt_prio1.json
python tools/wg_trace_summary.py $O/wgt_prio0.json $O/wgt_prio1.json > $O/wgt_prio_summary.jsonl
