#!/bin/bash
# Rotating A/B/C... of library builds on one box.  LIBS: space-separated list
# of library paths ("base" = the in-tree build); WORK: "headline" (bench.py)
# or "ragged" (bench_workloads.py --workload ragged); ROUNDS rotations.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-3}); do
  for lib in $LIBS; do
    if [ $lib = base ]; then unset MH_LIB_PATH; else export MH_LIB_PATH=$lib; fi
    tag=$(basename $lib .so)
    if [ "$WORK" = ragged ]; then
      timeout -k 10 200 python bench_workloads.py --workload ragged --steps ${STEPS:-20} --no-check > gpurun_out/abm.json 2> gpurun_out/abm.err || { tail -5 gpurun_out/abm.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/abm.json')); print('ragged $tag', d['value'], d['ms_per_step'], d['kernel_ms']['entries_varlen'], d['sha']['frac'])"
    else
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-1000} > gpurun_out/abm.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/abm.json')); print('headline $tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['sha']['frac'], d['single_build']['ms_per_build'])"
    fi
  done
done
