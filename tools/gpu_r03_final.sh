#!/bin/bash
# Last validation box of round 3: every -m gpu test, smoke(), the bench's default
# and the driver's command, the a14 bench line, then rocprofv3 --kernel-trace
# --stats of the default command (split by tools/prof_summary.py).
set -eo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 600 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
timeout -k 10 300 python bench_workloads.py --workload txlog --steps 200 > $O/bench_txlog.json 2> $O/bench_txlog.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 2000 --warmup 3 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/trace.log
python3 $R/tools/prof_summary.py $(find $O/trace -name "*kernel_trace.csv") --steps 2000 --warmup 3 > $O/summary.json
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/trace -name "*kernel_trace.csv" -exec gzip -c {} \; > $O/kernel_trace.csv.gz
rm -rf $O/trace
