set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wl
for w in c3 c5 ragged wire txlog; do
  timeout -k 10 300 python -u bench_workloads.py --workload $w > gpurun_out/wl/$w.json 2> gpurun_out/wl/$w.err || exit 1
done
