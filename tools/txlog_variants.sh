cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04k
for v in base MH_TXLOG_FUSED=0 MH_TXLOG_E=1 MH_TXLOG_KERNEL=group; do
  envs=""; [ "$v" != base ] && envs="$v"
  env $envs timeout -k 10 300 python bench_workloads.py --workload txlog > gpurun_out/r04k/$v.json 2> gpurun_out/r04k/$v.err || { tail -5 gpurun_out/r04k/$v.err; exit 1; }
  echo "$v $(tail -1 gpurun_out/r04k/$v.json)" | tee -a gpurun_out/r04k/all.txt
done
