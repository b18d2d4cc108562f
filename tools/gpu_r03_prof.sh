#!/bin/bash
# Round 3 profiles of the headline: rocprofv3 --kernel-trace --stats of the
# bench's default command (summary split by tools/prof_summary.py), then the two
# PMC traffic passes of the dominant kernel (separate runs, --kernel-trace only
# beside --pmc).
set -eo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r03b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 2000 --warmup 3 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/trace.log
python3 $R/tools/prof_summary.py $(find $O/trace -name "*kernel_trace.csv") --steps 2000 --warmup 3 > $O/summary.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 3 --warmup 1 --prewarm 0 --no-cpu-baseline > $O/pmc_$c.log 2>&1
done
python3 $R/tools/traffic_json.py $O "k_entries_fixed" "k_entries_fixed<2>" 1140850688 > $O/traffic.json
