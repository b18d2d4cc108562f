#!/bin/bash
# Group commit A/B on one box: the in-tree library (committers copy their own
# txs into the open batch's arena and their results out) vs build/ab/old (the
# worker packs and scatters every tx), interleaved, over batch caps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/queue_ab.txt
for r in 1 2; do
  for mt in 15 64; do
    for v in new old; do
      if [ $v = old ]; then LP=build/ab/old; else LP=immustore_amd; fi
      LD_LIBRARY_PATH=$LP timeout -k 10 120 tools/queue_bench 30 2000 16 1024 20 $mt > gpurun_out/q.json || exit 1
      python3 -c "import json,sys; d=json.load(open('gpurun_out/q.json')); g=d['gpu']; print('$v', 'max_txs', $mt, g['txs_per_s'], g['p50_us'], g['p99_us'], g['mean_batch_txs'], d['eh_match'])" >> gpurun_out/queue_ab.txt
    done
  done
done
cat gpurun_out/queue_ab.txt
