#!/bin/bash
# A/B of protobuf-writer library variants (built with EXTRA_FLAGS=-D... into
# build/lib_*.so): bash tools/pb_ab.sh build/lib_x.so ...  ("" = in-tree library), 2 rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
for lib in "" "$@"; do
  MH_LIB_PATH=$lib timeout -k 10 200 python -u bench_workloads.py --workload wire > gpurun_out/pb_ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/pb_ab.json'));print('${lib:-default}', d['kernel_ms'], d['inclusion_proof_pb']['kernel_ms'], d['sample_vs_oracle'])"
done
done
