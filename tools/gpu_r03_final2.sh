#!/bin/bash
# Round 3 closing box: tools/gpu_r03_final.sh (every -m gpu test, smoke, bench
# default + driver command, a14 line, rocprofv3 stats) and then every bench
# line on the same box (tools/bench_all.sh).
set -eo pipefail
bash "$GRAFT_REPO_ROOT/tools/gpu_r03_final.sh"
bash "$GRAFT_REPO_ROOT/tools/bench_all.sh"
