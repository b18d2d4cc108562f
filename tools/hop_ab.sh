# tx-log validation A/B by host hop thread count (MH_HOP_THREADS, read at run time)
# usage on the box: bash tools/hop_ab.sh  -> gpurun_out/hopab.log
set -e
for t in 8 16 12 16 8; do
  echo "threads=$t" >> gpurun_out/hopab.log
  MH_HOP_THREADS=$t timeout -k 10 120 python bench_workloads.py --workload txlog --steps 30 --warmup 3 >> gpurun_out/hopab.log 2>&1
done
