#!/bin/bash
# GPU validation pass: smoke -> parity tests -> bench -> kernel trace.
# Stops at the first crash/timeout (rc other than 0/1); test failures (rc 1)
# still let the bench run so one box call yields both pictures.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/smoke.log | tail -5
[ $rc -gt 1 ] && exit $rc
timeout -k 10 1200 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; grep -v amdgpu.ids gpurun_out/bench.err | tail -5
[ $rc -ne 0 ] && exit $rc
if [ -n "$WORKLOADS" ]; then
  for w in $WORKLOADS; do
    timeout -k 10 300 python bench_workloads.py --workload $w > gpurun_out/w_$w.json 2> gpurun_out/w_$w.err || { grep -v amdgpu.ids gpurun_out/w_$w.err | tail -5; exit 1; }
    cat gpurun_out/w_$w.json
  done
fi
[ -n "$NO_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
# the default bench command (same steps / warmup / builds in flight) under the profiler
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?
grep '^{"metric"' "$GRAFT_REPO_ROOT/gpurun_out/prof.log" > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json"
python3 "$GRAFT_REPO_ROOT/tools/prof_summary.py" "$GRAFT_REPO_ROOT/gpurun_out/prof/run_kernel_trace.csv" --steps 2000 --warmup 3 | tee "$GRAFT_REPO_ROOT/gpurun_out/prof_summary.json"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*"
exit $rc
