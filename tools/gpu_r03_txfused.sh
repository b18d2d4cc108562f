#!/bin/bash
# a14 with one fused launch per small-tree group (k_txlog_group, default; without
# the L2 warm-up of the records: MH_TXLOG_WARM=0) vs the six-launch chain
# (MH_TXLOG_FUSED=0): tx-log parity first, then an
# interleaved bench_workloads txlog A/B.  -> profiles/ab_txlog_fused_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tx.py tests/test_gpu_concurrency.py tests/test_gpu_c_client.py tests/test_gpu_commit.py > $O/pytest_txfused.log 2>&1
: > $O/txfused_ab.txt
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench_workloads.py --workload txlog --steps 200 > $O/tf.json 2>/dev/null
  echo "$n $(python3 -c "import json;d=json.loads(open('$O/tf.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['pageable_input']['ms_per_step'],d['host_hop_only_ms'],{k:v for k,v in d['kernel_ms'].items() if v})")" >> $O/txfused_ab.txt
}
for r in $(seq ${ROUNDS:-3}); do
  run ${V1:-fused} ${E1:-MH_DUMMY=1}
  run ${V2:-fused_nowarm} ${E2:-MH_TXLOG_WARM=0}
  run ${V3:-chain} ${E3:-MH_TXLOG_FUSED=0}
done
cp $O/tf.json $O/bench_txlog_fused.json
cat $O/txfused_ab.txt
