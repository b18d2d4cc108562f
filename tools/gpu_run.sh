#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_r0*_*.sh
# wrappers).  Usage, as a gpurun command:
#   TAG=r04a tools/gpu_run.sh tests smoke bench bench_cabi corrupt c3cabi dist2 prof
# Each named step runs under its own time limit, writes gpurun_out/$TAG/<step>.*
# and the runner stops at the first failing step (no GPU step after a fault).
# Steps:
#   tests            every -m gpu test            tests:<expr>  only -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            the driver's default command (python bench.py)
#   bench_cabi       bench.py --api cabi --gpus 1 (one-device RCCL clique)
#   corrupt          bench.py with MH_BENCH_CORRUPT=0: must exit 1 (root check)
#   corrupt_cabi     the same through --api cabi
#   c3cabi           bench.py --api cabi --config c3 (replay append onto n0)
#   dist2            2 gloo ranks sharing GPU 0 (bench.py --gpus 2 rehearsal)
#   c4               bench.py --config c4 (2^23 x 4 KiB, sampled root check)
#   prof             rocprofv3 --kernel-trace --stats of the driver bench
#   txlog            tools/txlog_bench (a14 through the C ABI)
#   workloads        bench_workloads.py: every secondary workload line
#   ab:<VARIANTS>    tools/ab_env.sh rotation, e.g. ab:base,MH_LPL=1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p "$O"
B="timeout -k 10"
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  $B "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  tail -3 "$O/$name.out"
  grep -v amdgpu.ids "$O/$name.err" | tail -3
  return $rc
}
for s in "$@"; do
  case "$s" in
    tests) step tests 1100 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/ || exit 1 ;;
    tests:*) step tests_k 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/ -k "${s#tests:}" || exit 1 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1 ;;
    bench) step bench 400 python bench.py || exit 1 ;;
    bench_cabi) step bench_cabi 300 python bench.py --api cabi --gpus 1 --steps 200 --warmup 5 || exit 1 ;;
    corrupt)
      MH_BENCH_CORRUPT=0 step corrupt 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
      rc=$?; echo "corrupt exit $rc (want 1)"; [ $rc -eq 1 ] || exit 1 ;;
    corrupt_cabi)
      MH_BENCH_CORRUPT=0 step corrupt_cabi 300 python bench.py --api cabi --gpus 1 --steps 20 --warmup 3
      rc=$?; echo "corrupt_cabi exit $rc (want 1)"; [ $rc -eq 1 ] || exit 1 ;;
    c3cabi) step c3cabi 400 python bench.py --api cabi --gpus 1 --config c3 --steps 10 --warmup 2 || exit 1 ;;
    dist2)
      MH_DIST_BACKEND=gloo HIP_VISIBLE_DEVICES=0 step dist2 400 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
        bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1 ;;
    c4) step c4 600 python bench.py --config c4 --steps 5 --warmup 1 --prewarm 0 --no-cpu-baseline || exit 1 ;;
    prof)
      rm -rf "$O/prof"
      step prof 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1 ;;
    txlog) step txlog 300 ./tools/txlog_bench || exit 1 ;;
    workloads) step workloads 900 bash tools/bench_all.sh || exit 1 ;;
    ab:*) VARIANTS="$(echo "${s#ab:}" | tr ';' ' ')" step ab 900 bash tools/ab_env.sh || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== all steps ok"
