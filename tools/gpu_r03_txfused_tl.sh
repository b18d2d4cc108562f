#!/bin/bash
# a14 timeline, fused group kernel (default) vs the six-launch chain
# (MH_TXLOG_FUSED=0): MH_TXLOG_TRACE phase stamps of plain runs, then a kernel +
# memory-copy trace of each (no counters), last call summarised by
# tools/trace_window.py.  -> profiles/txlog_fused_timeline_r03.txt
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for r in 1 2 3; do
  MH_TXLOG_TRACE=1 timeout -k 10 120 python tools/txlog_timeline.py > $O/tl_fused_plain$r.txt 2>&1
  MH_TXLOG_FUSED=0 MH_TXLOG_TRACE=1 timeout -k 10 120 python tools/txlog_timeline.py > $O/tl_chain_plain$r.txt 2>&1
done
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/txtl_f -o run -- python3 tools/txlog_timeline.py > $O/tl_fused_prof.txt 2>&1
python3 tools/trace_window.py $O/txtl_f 2500 > $O/tl_fused_window.txt
MH_TXLOG_FUSED=0 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/txtl_c -o run -- python3 tools/txlog_timeline.py > $O/tl_chain_prof.txt 2>&1
python3 tools/trace_window.py $O/txtl_c 2500 > $O/tl_chain_window.txt
rm -rf $O/txtl_f $O/txtl_c
