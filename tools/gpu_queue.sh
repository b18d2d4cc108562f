#!/bin/bash
# Group commit (tools/queue_bench) over worker counts, gather windows and
# batch caps (MAXTXS; a cap below the committer count lets two batches be in
# flight in a closed loop):
# one JSON line per run (with "workers") into gpurun_out/queue_bench.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/queue_bench.jsonl
for w in ${WORKERS:-1 2}; do
  for wu in ${WAITS:-0 20 50}; do
   for mt in ${MAXTXS:-64}; do
    MH_QUEUE_WORKERS=$w timeout -k 10 120 tools/queue_bench 30 2000 16 1024 $wu $mt > gpurun_out/q.json || exit 1
    python3 - "$w" >> gpurun_out/queue_bench.jsonl <<'PY'
import json, sys
d = json.load(open("gpurun_out/q.json"))
d["workers"] = int(sys.argv[1])
print(json.dumps(d))
PY
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/queue_bench.jsonl')][-1]; g=d['gpu']; print(d['workers'], d['wait_us'], d.get('max_txs'), g['txs_per_s'], g['p50_us'], g['p99_us'], g['mean_batch_txs'], d['eh_match'])"
   done
  done
done
