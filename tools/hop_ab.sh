cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for lib in "" build/lib_t16.so build/lib_t4.so; do
  MH_LIB_PATH=$lib timeout -k 10 120 python -u bench_workloads.py --workload txlog > gpurun_out/hop_ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hop_ab.json'));print('${lib:-t8}', d['ms_per_step'], d['pageable_input']['ms_per_step'])"
done; done
