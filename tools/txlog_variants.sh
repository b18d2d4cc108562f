#!/bin/bash
# bench_workloads.py --workload txlog under env variants (default: the a14 kernel
# variants): end-to-end ms per call and the call's hashing-kernel time.
# usage: txlog_variants.sh [VARIANT ...]   (VARIANT = base or NAME=VALUE[,NAME=VALUE])
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04k}
mkdir -p $O
vs="$*"
[ -z "$vs" ] && vs="base MH_TXLOG_FUSED=0 MH_TXLOG_E=1 MH_TXLOG_KERNEL=group"
for v in $vs; do
  envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench_workloads.py --workload txlog > $O/wl.json 2> $O/wl.err || { tail -5 $O/wl.err; exit 1; }
  echo "$v $(tail -1 $O/wl.json)" | tee -a $O/all.txt
done
