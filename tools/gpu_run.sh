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
#   txcabi           bench.py --api cabi --config txlog (mh_multi_txlog_validate); txcabi_corrupt: must exit 1
#   dist2            2 gloo ranks sharing GPU 0 (bench.py --gpus 2 rehearsal)
#   dist8            8 gloo ranks sharing GPU 0 (the driver's N = 8 path rehearsed)
#   dist2s / dist8s  the same with --scaling strong (one 2^20 tree split over the ranks);
#                    dist8s_corrupt: rank 5 corrupted, must exit 1; strong1: N = 1 strong
#   committers       tests/c_client/mh_committers: threads x clique-pool sizes -> committers.txt
#   lanes_check      rebuild with LANES_CHECK=1 (range-checked lanes kernel), then the tx-log tests
#   c4               bench.py --config c4 (2^23 x 4 KiB, sampled root check)
#   wdist:<w>:<N>    bench_workloads.py --workload <w> (c3 / c5) as N gloo ranks sharing GPU 0
#   wcorrupt:<w>:<N> the same with MH_BENCH_CORRUPT=1 (N >= 2): must exit 1 (result check)
#   pgprof:<VARS>    rocprofv3 kernel trace of bench.py per env variant -> queue map + overlap
#   forcepg          MH_DIST_FORCE_PG=1: the multi-rank code paths as ONE nccl (RCCL) rank:
#                    bench.py (C2), bench.py --config c4, bench_workloads.py c3 and c5
#   prof             rocprofv3 --kernel-trace --stats of the driver bench
#   txlog            tools/txlog_bench (a14 through the C ABI)
#   txclog           tools/txlog_bench with TXB_CLOG=1 (mh_txlog_validate_clog, pinned log + cLog)
#   waveprobe        k_txlog_wave per-phase stamps of the a14 call's last group (make WAVE_PROBE=1 build)
#   txwl             bench_workloads.py --workload txlog (a14 + resident / cLog lines) -> txwl.out
#   copyprobe        tools/copy_probe: chunked pinned H2D pipeline costs (host wall time)
#   workloads        bench_workloads.py: every secondary workload line
#   ab:<VARIANTS>    tools/ab_env.sh rotation, e.g. ab:base,MH_LPL=1
#   txab:<VARIANTS>  tools/txlog_bench rotation (ROUNDS x), e.g. txab:base;MH_TXLOG_KERNEL=lanes
#   txtl:<VARIANTS>  a14 kernel + copy timeline of the last call per variant -> txtl.txt
#   workload:<name>  bench_workloads.py --workload <name>
#   txres:<VARS>     a14 kernel over a resident log (tools/txlog_resident.py) per env variant
#   fuzz             host-ASan tx-log fuzzer with the device path (FUZZ_ITERS, FUZZ_SEED)
#   queue            tools/queue_bench: group commit, 30 committers (QWAIT us, QMAXTXS)
#   traffic          tools/gpu_pmc.sh: the counter passes behind traffic_r*.json (PMC_CMD overrides)
#   pmctx            tools/gpu_pmc_txlog.sh (PMC_MATCH=kernel name) -> gpurun_out/pmctx/table.txt
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
    txcabi) step txcabi 400 python bench.py --api cabi --gpus 1 --config txlog --steps 100 --warmup 5 --prewarm 1 || exit 1 ;;
    txcabi_corrupt)
      MH_BENCH_CORRUPT=0 step txcabi_corrupt 400 python bench.py --api cabi --gpus 1 --config txlog --steps 5 --warmup 1 --prewarm 0
      rc=$?; echo "txcabi_corrupt exit $rc (want 1)"; [ $rc -eq 1 ] || exit 1 ;;
    c3cabi) step c3cabi 400 python bench.py --api cabi --gpus 1 --config c3 --steps 10 --warmup 2 || exit 1 ;;
    dist2)
      MH_DIST_BACKEND=gloo HIP_VISIBLE_DEVICES=0 step dist2 400 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
        bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1 ;;
    dist8)  # 8 gloo ranks sharing GPU 0: the driver's N = 8 path (root check over 8 ranks) rehearsed
      MH_DIST_BACKEND=gloo HIP_VISIBLE_DEVICES=0 step dist8 500 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 \
        bench.py --gpus 8 --steps 20 --warmup 3 --prewarm 1 --no-cpu-baseline || exit 1 ;;
    dist2s|dist8s)  # --scaling strong: ONE 2^20-entry tree over N gloo ranks sharing GPU 0 (root vs the oracle)
      n=${s:4:1}
      MH_DIST_BACKEND=gloo HIP_VISIBLE_DEVICES=0 step "$s" 500 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 2953$n \
        bench.py --gpus "$n" --scaling strong --steps 20 --warmup 3 --prewarm 1 --no-cpu-baseline || exit 1 ;;
    dist8s_corrupt)  # the same with rank 5's shard corrupted: must exit 1
      MH_BENCH_CORRUPT=5 MH_DIST_BACKEND=gloo HIP_VISIBLE_DEVICES=0 step dist8s_corrupt 500 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29539 \
        bench.py --gpus 8 --scaling strong --steps 5 --warmup 1 --prewarm 0 --no-cpu-baseline
      rc=$?; echo "dist8s_corrupt exit $rc (want 1)"; [ $rc -eq 1 ] || exit 1 ;;
    lanes_check)  # the range-checking k_txlog_lanes (make LANES_CHECK=1, built here over the snapshot's
      # library) under every tx-log test: any read outside the log fails the call
      step lanes_build 600 make -s -j16 -C immustore_amd/csrc LANES_CHECK=1 || exit 1
      step lanes_check 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/ \
        -k "txlog or clog or resident or fused or c_client" || exit 1 ;;
    committers)  # concurrent committers over a clique pool (tests/c_client/mh_committers): aggregate
      # GiB/s of values per (threads, cliques), 3 interleaved rounds
      for r in 1 2 3; do
        for tc in "2 1" "2 2" "4 1" "4 2" "4 4"; do
          set -- $tc
          line=$(timeout -k 10 120 tests/c_client/mh_committers $1 $2 ${CM_ROUNDS:-10} ${CM_NTX:-4096} 16 1024 | grep '^rate') || exit 1
          echo "round $r threads $1 cliques $2 $line" | tee -a "$O/committers.txt"
        done
      done ;;
    strong1) step strong1 300 python bench.py --scaling strong --steps 200 --warmup 5 --no-cpu-baseline || exit 1 ;;
    wdist:*|wcorrupt:*)  # bench_workloads.py multi-rank lines, N gloo ranks sharing GPU 0
      w=$(echo "$s" | cut -d: -f2); n=$(echo "$s" | cut -d: -f3); kind=${s%%:*}
      corrupt=""; [ "$kind" = wcorrupt ] && corrupt="MH_BENCH_CORRUPT=1"
      env $corrupt MH_DIST_BACKEND=gloo HIP_VISIBLE_DEVICES=0 timeout -k 10 600 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29541 \
        bench_workloads.py --workload "$w" --steps 5 --warmup 1 > "$O/${kind}_${w}_$n.out" 2> "$O/${kind}_${w}_$n.err"
      rc=$?; tail -2 "$O/${kind}_${w}_$n.out"; grep -v amdgpu.ids "$O/${kind}_${w}_$n.err" | grep -i "fail\|error" | tail -2
      if [ "$kind" = wcorrupt ]; then echo "$s exit $rc (want 1)"; [ $rc -eq 1 ] || exit 1
      else [ $rc -eq 0 ] || exit 1; fi ;;
    forcepg)  # the torch.distributed / RCCL code paths executed as one nccl rank
      MH_DIST_FORCE_PG=1 step forcepg_c2 400 python bench.py --steps 200 --warmup 5 --no-cpu-baseline || exit 1
      MH_DIST_FORCE_PG=1 step forcepg_c4 600 python bench.py --config c4 --steps 5 --warmup 1 --prewarm 0 --no-cpu-baseline || exit 1
      MH_DIST_FORCE_PG=1 step forcepg_wc3 600 python bench_workloads.py --workload c3 --steps 5 --warmup 1 || exit 1
      MH_DIST_FORCE_PG=1 step forcepg_wc5 600 python bench_workloads.py --workload c5 --steps 5 --warmup 1 || exit 1 ;;
    pgprof:*)  # kernel traces of bench.py per env variant (e.g. pgprof:base;MH_DIST_FORCE_PG=1) -> queue map
      vs="$(echo "${s#pgprof:}" | tr ';' ' ')"; i=0
      for v in $vs; do
        i=$((i+1)); envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
        rm -rf "$O/pgprof_$i"
        env $envs timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/pgprof_$i" -o run -- python3 bench.py --steps ${PG_STEPS:-200} --warmup 5 --no-cpu-baseline > "$O/pgprof_$i.out" 2> "$O/pgprof_$i.err" || { tail -5 "$O/pgprof_$i.err"; exit 1; }
        { echo "# variant $v: $(tail -1 "$O/pgprof_$i.out" | cut -c1-160)"; python3 tools/queue_map.py "$O/pgprof_$i"; } | tee -a "$O/pgprof.txt"
        rm -rf "$O/pgprof_$i"
      done ;;
    c4) step c4 600 python bench.py --config c4 --steps 5 --warmup 1 --prewarm 0 --no-cpu-baseline || exit 1 ;;
    prof)
      rm -rf "$O/prof"
      step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
      python3 tools/prof_summary.py "$O/prof/run_kernel_trace.csv" --steps 20 --warmup 5 > "$O/prof_summary.json" || exit 1
      gzip -f "$O/prof/run_kernel_trace.csv" ;;
    txlog) step txlog 300 ./tools/txlog_bench || exit 1 ;;
    txclog) TXB_CLOG=1 step txclog 300 ./tools/txlog_bench ${TXB_ARGS:-200} || exit 1 ;;
    waveprobe) step waveprobe_build 600 make -s -j16 -C immustore_amd/csrc WAVE_PROBE=1 || exit 1
      step waveprobe 300 python tools/txlog_wave_probe.py || exit 1 ;;
    txwl) step txwl 400 python bench_workloads.py --workload txlog --steps ${TXWL_STEPS:-50} --warmup 3 || exit 1 ;;
    copyprobe) step copyprobe 200 ./tools/copy_probe || exit 1 ;;
    workloads) step workloads 900 bash tools/bench_all.sh || exit 1 ;;
    txab:*)  # interleaved A/B of tools/txlog_bench over env variants, e.g. txab:base;MH_TXLOG_KERNEL=lanes
      vs="$(echo "${s#txab:}" | tr ';' ' ')"
      for i in $(seq ${ROUNDS:-3}); do
        for v in $vs; do
          envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
          env $envs timeout -k 10 200 ./tools/txlog_bench ${TXB_ARGS:-200} > "$O/txab.json" 2> "$O/txab.err" || { cat "$O/txab.err"; exit 1; }
          echo "$v $(cat "$O/txab.json")" | tee -a "$O/txab.txt"
        done
      done ;;
    txtl:*)  # a14 timeline per env variant: kernel + memory-copy trace of the last call (tools/trace_window.py)
      vs="$(echo "${s#txtl:}" | tr ';' ' ')"
      for v in $vs; do
        envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
        rm -rf "$O/txtl"
        api=""; [ -n "${TXTL_API:-}" ] && api="--hip-runtime-trace"  # TXTL_API=1: host HIP calls too
        env $envs timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace $api --output-format csv -d "$O/txtl" -o run -- python3 tools/txlog_timeline.py > "$O/txtl.out" 2>&1 || { tail -5 "$O/txtl.out"; exit 1; }
        { echo "# variant $v"; python3 tools/trace_window.py "$O/txtl" 2500; } | tee -a "$O/txtl.txt"
      done
      rm -rf "$O/txtl" ;;
    fuzz)  # host-ASan tx-log fuzzer with the device path (tools/asan/; built on the box, ~30 s)
      { [ -x build/asan/txlog_fuzz ] || make -s -j16 -C tools/asan > "$O/asan_build.log" 2>&1; } || { tail -5 "$O/asan_build.log"; exit 1; }
      python3 tools/asan/make_corpus.py "$O/corpus" > /dev/null || exit 1
      ASAN_OPTIONS=detect_leaks=0 MH_FUZZ_DEVICE=1 step fuzz ${FUZZ_TIMEOUT:-500} \
        build/asan/txlog_fuzz ${FUZZ_ITERS:-2000} ${FUZZ_SEED:-20261016} "$O"/corpus/*.log
      rc=$?; rm -rf "$O/corpus"; [ $rc -eq 0 ] || exit 1 ;;
    queue) step queue 300 ./tools/queue_bench 30 2000 16 1024 ${QWAIT:-20} ${QMAXTXS:-64} || exit 1 ;;
    traffic) step traffic 1200 bash tools/gpu_pmc.sh || exit 1 ;;
    txres:*)  # a14 kernel over a resident log per env variant (tools/txlog_resident.py) -> txres.txt
      vs="$(echo "${s#txres:}" | tr ';' ' ')"
      for v in $vs; do
        envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
        env $envs timeout -k 10 200 python3 tools/txlog_resident.py ${TXRES_ARGS:-} > "$O/txres.out" 2> "$O/txres.err" || { tail -5 "$O/txres.err"; exit 1; }
        { echo "# variant $v: $(tail -1 "$O/txres.out")"; grep txlog_probe "$O/txres.err" | tail -2; } | tee -a "$O/txres.txt"
      done ;;
    workload:*) w="${s#workload:}"; step "wl_$w" 600 python bench_workloads.py --workload "$w" || exit 1 ;;
    pmctx) step pmctx 900 bash tools/gpu_pmc_txlog.sh || exit 1; cat "gpurun_out/pmctx${PMC_TAG:-}/table.txt" ;;
    ab:*) VARIANTS="$(echo "${s#ab:}" | tr ';' ' ')" step ab 900 bash tools/ab_env.sh || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== all steps ok"
