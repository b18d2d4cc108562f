#!/bin/bash
# a14 timeline: kernel + memory-copy trace of the last mh_txlog_validate call
# (no counters), summarised by tools/trace_window.py; plain timings with the
# copies issued inline (default for a pinned log) and from the helper thread.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tx.py -k txlog > $O/pytest_tx.log 2>&1
for r in 1 2; do
  timeout -k 10 120 python tools/txlog_timeline.py > $O/txlog_timeline_plain_inl$r.txt 2>&1
  MH_TXLOG_INLINE_COPY=0 timeout -k 10 120 python tools/txlog_timeline.py > $O/txlog_timeline_plain_thr$r.txt 2>&1
done
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/txtl -o run -- python3 tools/txlog_timeline.py > $O/txlog_timeline_prof.txt 2>&1
python3 tools/trace_window.py $O/txtl 2500 > $O/txlog_timeline_window.txt
