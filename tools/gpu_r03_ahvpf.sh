#!/bin/bash
# ahtree proof re-hash compiled per kind (inclusion kinds at ~60 VGPRs instead of
# 123, next term loaded under the current hash) vs the one-kernel-for-all-kinds
# build (build_ab/base.so): ahtree / dual-proof / document parity first, then an
# interleaved c5 A/B (htree + ahtree inclusion + consistency lines).
# -> profiles/ab_ahtree_verify_kinds_r03.txt
set -eo pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_tx.py tests/test_gpu_pb_decode.py \
  -k "verify or c5 or proof or dual or document" > $O/pytest_ahvpf.log 2>&1
: > $O/ahvpf_ab.txt
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench_workloads.py --workload c5 > $O/c5a.json 2>/dev/null
  echo "$n $(python3 -c "import json;d=json.loads(open('$O/c5a.json').read().strip().splitlines()[-1]);a=d['ahtree'];print(d['value'],a['inclusion']['M_proofs_per_s'],a['consistency']['M_proofs_per_s'])")" >> $O/ahvpf_ab.txt
}
for r in 1 2 3; do
  run kinds MH_DUMMY=1
  run base MH_LIB_PATH=$PWD/build_ab/base.so
done
cat $O/ahvpf_ab.txt
