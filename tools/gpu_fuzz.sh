#!/bin/bash
# Host-ASan tx-log fuzzer with the device path (MH_FUZZ_DEVICE=1): every mutant
# through mh_txlog_scan, mh_txlog_validate and the oracle (tools/asan/).
# build/asan is not sent to the box (.gpurunignore): built there first (~30 s).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
[ -x build/asan/txlog_fuzz ] || make -s -j16 -C tools/asan > gpurun_out/asan_build.log 2>&1 || { tail -5 gpurun_out/asan_build.log; exit 1; }
python3 tools/asan/make_corpus.py gpurun_out/corpus > /dev/null || exit 1
ASAN_OPTIONS=detect_leaks=0 MH_FUZZ_DEVICE=1 timeout -k 10 ${FUZZ_TIMEOUT:-500} \
  build/asan/txlog_fuzz ${FUZZ_ITERS:-2000} ${FUZZ_SEED:-20261016} gpurun_out/corpus/*.log \
  > gpurun_out/fuzz_device.log 2>&1; rc=$?
rm -rf gpurun_out/corpus
cat gpurun_out/fuzz_device.log | tail -20
exit $rc
