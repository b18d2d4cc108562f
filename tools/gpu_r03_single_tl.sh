#!/bin/bash
# kernel timeline of single C2 builds (no timing events)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 120 python tools/single_build_timeline.py > $O/single_plain.txt 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/sbtl -o run -- python3 tools/single_build_timeline.py > $O/single_prof.txt 2>&1
python3 tools/trace_window.py $O/sbtl 2000 > $O/single_window.txt
