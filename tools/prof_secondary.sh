#!/bin/bash
# rocprofv3 kernel-trace summaries of the secondary workloads (8(f) rows 3/4,
# a14): protobuf proof writers, c3 with appendable records, tx-log validation.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
for w in "wire" "c3 --logs" "txlog"; do
  tag=$(echo "$w" | tr -d ' -')
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2/$tag -o run \
    -- python3 bench_workloads.py --workload $w > gpurun_out/prof2/$tag.json 2> gpurun_out/prof2/$tag.err || exit 1
done
