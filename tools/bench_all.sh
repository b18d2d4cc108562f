#!/bin/bash
# Every benchmark line of the round on one box: bench.py (headline, c4) and
# bench_workloads.py (c3, c3 --logs, c3range, c5, c2e2e, txlog, commit, wire, ragged,
# document, values), then one JSON line per run in gpurun_out/all/all.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/all
timeout -k 10 300 python -u bench.py > gpurun_out/all/c2.json 2> gpurun_out/all/c2.err || exit 1
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/all/c4.json 2> gpurun_out/all/c4.err || exit 1
for w in c3 "c3 --logs" c3range c5 c2e2e txlog commit wire ragged document values; do
  tag=$(echo "$w" | tr -d ' -')
  timeout -k 10 300 python -u bench_workloads.py --workload $w > gpurun_out/all/$tag.json 2> gpurun_out/all/$tag.err || exit 1
done
for f in gpurun_out/all/*.json; do tail -n 1 "$f"; done > gpurun_out/all/all.jsonl
