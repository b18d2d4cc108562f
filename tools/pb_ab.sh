#!/bin/bash
# A/B of the staged protobuf writers' records-per-round (library variants built
# with EXTRA_FLAGS=-DMH_PB_RPR=n into build/lib_r<n>.so), 2 rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
for lib in "" build/lib_r8.so; do
  MH_LIB_PATH=$lib timeout -k 10 200 python -u bench_workloads.py --workload wire > gpurun_out/pb_ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/pb_ab.json'));print('${lib:-rpr4}', d['kernel_ms'], d['inclusion_proof_pb']['kernel_ms'], d['sample_vs_oracle'])"
done
done
