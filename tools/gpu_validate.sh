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
[ -n "$NO_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?
tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*"
exit $rc
