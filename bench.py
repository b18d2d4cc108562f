#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on MI355X.

metric: device-resident GiB/s hashed, htree build, 1M x 1 KiB leaves.

One "step" = one full htree build over one batch of entries already resident
in HBM (BASELINE configs[1]): for every entry hVal = SHA256(value) (1 KiB),
the v1 entry digest, the leaf hash, and every level of the tree up to the
root (embedded/store/immustore.go:1620-1632, tx.go:332-355, htree.go:68-113),
all by the HIP kernels of libimmustore_merkle.so through its C ABI.

--gpus N (launched by torch.distributed.run, one process per GPU): every rank
builds the subtree over its own 2^20 entries (power-of-two aligned shard of a
global N x 2^20-leaf tree), the N subtree roots are all-gathered over RCCL and
the top log2(N) levels are reduced on every rank (exact by
finding 3).  Weak scaling by default: per-GPU work is fixed (the metric's
"1M x 1KiB leaves @1/2/4/8 GPU" read as 1M leaves per GPU, an N x 2^20-leaf
tree).  --scaling strong reads it as ONE 2^20 x 1 KiB tree at every N: each
rank builds 2^20 / N leaves (power-of-two N: shards stay aligned subtrees),
the values being exactly the N = 1 tree's (the splitmix64 stream at the
rank's entry offset), so the root is the same at every N.

--config c4 runs BASELINE configs[3] instead: 2^23 x 4 KiB entries per GPU
(values generated in HBM), i.e. the 2^26-entry tree at 8 GPUs.

--api cabi runs the same sharded build from ONE process driving N devices
through the C ABI a cgo caller would use (mh_multi_create over devices
0..N-1: one context per device and the library's own RCCL clique,
mh_multi_dev_htree_build_entries_fixed per step), instead of N
torch.distributed ranks.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

N_ENTRIES = 1 << 20
VAL_LEN = 1024
KEY_LEN = 8
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU instructions per 64-byte compression of the generic compress() in the
# gfx950 ISA of this build (counted in profiles/isa_counts_r01.txt); the
# constant-schedule padding block (compress_kw) needs fewer.
OPS_PER_COMP = 1388
OPS_PER_COMP_KW = 901
# Measured SHA-256 compression ceiling of this chip with this round function:
# tools/microbench_sha.hip, registers only, 8 waves/SIMD, 30.9 G compressions/s
# (profiles/microbench_r01.txt, line "waves/SIMD 8").
SHA_PEAK_GCOMPS = 30.9
# VALU peak FOR THIS INSTRUCTION MIX (lane-ops/s): the measured compression
# ceiling above x the 1388 VALU instructions of one compression x 64 lanes / 64
# (one wave-instruction = 64 lane-ops per compression lane) = 42.9 T.  Not the
# nominal 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T: on gfx950
# v_alignbit_b32 and v_add3_u32 -- 805 of the 1388 -- issue at 1.93 / 2.04 ns
# per wave-instruction per SIMD against 1.26-1.33 for add / xor / bitop3
# (profiles/microbench_r01.txt, microbench_valu rows), so no SHA-256 round
# reaches the nominal figure.
VALU_PEAK_OPS = SHA_PEAK_GCOMPS * 1e9 * OPS_PER_COMP


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--prewarm", type=float, default=5.0,
                   help="seconds of untimed builds before the warmup steps, so the GPU "
                        "clock is at its sustained value when timing starts (0 = off); "
                        "5 s rather than 2 also spans a utilisation sampler's 5 s period, "
                        "which saw the round-3 runs' GPU idle")
    p.add_argument("--config", choices=["c2", "c4", "c3", "c5", "txlog"], default="c2",
                   help="c2: BASELINE configs[1], 2^20 x 1 KiB per GPU (headline); c4: "
                        "configs[3], 2^23 x 4 KiB per GPU (2^26 entries at 8 GPUs); c3: "
                        "configs[2] ahtree append of 10^7; c5: configs[4] proof re-hash "
                        "(c3 / c5: one GPU, GPU part from bench_workloads.py); txlog: "
                        "SURVEY 8(a) a14 through the C ABI (--api cabi only)")
    p.add_argument("--entries", type=int, default=None,
                   help="override entries per GPU (--api cabi --config c3: total appends)")
    p.add_argument("--n0", type=int, default=10 ** 6 + 3,
                   help="--api cabi --config c3: size of the tree the batch is appended onto")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--launch-check", action="store_true",
                   help="only bring up the N-rank process group (gloo, no GPU work) and print "
                        "its world size: tests the --gpus N launcher on a CPU host")
    p.add_argument("--timing-in-region", action="store_true",
                   help="per-kernel timing events on inside the timed region (A/B; by default "
                        "the contended kernel time comes from a separate pass after it)")
    p.add_argument("--inflight", type=int, default=None,
                   help="independent builds in flight on separate streams (1 = sequential; "
                        "default 3, and 2 cliques with --api cabi: 1249 GiB/s at 2, 1186 at 3, "
                        "1166 at 4, profiles/cabi_inflight_r05.txt)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="target CPU work of the cpu_baseline sample")
    p.add_argument("--api", choices=["torch", "cabi"], default="torch",
                   help="torch: one process per GPU over torch.distributed (driver default); "
                        "cabi: one process, mh_multi_* over N devices with the in-library "
                        "RCCL clique (the cgo caller's path)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                   help="weak: 2^20 entries per GPU (default); strong: one 2^20-entry tree "
                        "split over the N GPUs (c2 only, N a power of two)")
    p.add_argument("--traffic-file", default=os.path.join(HERE, "profiles", "traffic_r06.json"),
                   help="PMC-derived HBM bytes per launch of the dominant kernel (or missing): "
                        "the round's rocprofv3 --pmc passes (tools/gpu_pmc.sh)")
    return p.parse_args()


# ------------------------------------------------------------------ root check
# After the timed region every multi-GPU (and single-GPU) line proves its own
# result: the oracle (oracle/, the CPU restatement of htree.go:68-113 and
# tx.go:332-355 pinned by the Go-written stores) rebuilds each shard from the
# same splitmix64 stream and BE64 keys the devices generated, and the top
# levels over the shard roots; the device roots must equal it bit for bit.
# The oracle is the checker here, never the thing measured.
SPLITMIX_G = 0x9E3779B97F4A7C15
CHECK_BLOCK_BITS = 14      # sampled mode: 2^14-entry blocks = level-14 nodes
FULL_CHECK_BYTES = 2 << 30  # shards up to this many value bytes: rebuilt whole


def _oracle():
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle as orc
    orc.use_shani(True)
    return orc


def host_threads(share=1):
    """Host threads this process may use, split over `share` processes."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    return max(1, avail // max(share, 1))


def shard_seed(rank, n, val, strong):
    """The mh_dev_fill_random seed of rank's values: weak, an independent
    stream per rank (2 + rank); strong, the N = 1 tree's stream (seed 2) from
    the rank's first entry on, so the N shards are that one tree's values."""
    if not strong:
        return 2 + rank
    return (2 + (rank * n * val // 8) * SPLITMIX_G) & 0xFFFFFFFFFFFFFFFF


def shard_block(orc, seed, key0, e0, cnt, val):
    """Entries [e0, e0 + cnt) of a shard whose values came from
    mh_dev_fill_random(seed) and keys from mh_dev_fill_keys_be64(key0): the
    splitmix64 stream from word e0 * val / 8 (word w = mix(seed + (w+1) G))."""
    s = (seed + (e0 * val // 8) * SPLITMIX_G) & 0xFFFFFFFFFFFFFFFF
    vals = orc.fill_random(cnt * val, s).reshape(cnt, val)
    keys = np.frombuffer(np.arange(key0 + e0, key0 + e0 + cnt, dtype=">u8").tobytes(),
                         np.uint8).reshape(cnt, KEY_LEN)
    return keys, vals


def oracle_shard_root(orc, n, val, seed, key0, levels_dev, threads):
    """The oracle's root of one shard (v1 entries, keys BE64(key0 + i)).
    full: every entry rebuilt (C2: 1 GiB per shard).  sampled (C4, 32 GiB per
    shard): three 2^14-entry blocks rebuilt and compared with the device's
    level-14 nodes, and the levels above rebuilt by the oracle from those
    nodes.  -> (root, blocks_ok, mode)."""
    if n * val <= FULL_CHECK_BYTES or n <= (1 << CHECK_BLOCK_BITS):
        keys, vals = shard_block(orc, seed, key0, 0, n, val)
        _, _, r = orc.build_entries_fixed(1, keys, vals, nthreads=threads, want_levels=False)
        return r, True, "full"
    import immustore_amd as m
    b, B = CHECK_BLOCK_BITS, 1 << CHECK_BLOCK_BITS
    nb = -(-n // B)
    off = m.level_offset(n, b)
    nodes = levels_dev[off * 32:(off + nb) * 32].cpu().numpy().reshape(nb, 32)
    rng = np.random.default_rng(seed)
    picks = sorted({0, nb - 1, int(rng.integers(0, nb))})
    ok = True
    for i in picks:
        e0 = i * B
        keys, vals = shard_block(orc, seed, key0, e0, min(B, n - e0), val)
        _, _, r = orc.build_entries_fixed(1, keys, vals, nthreads=threads, want_levels=False)
        ok &= r == nodes[i].tobytes()
    r = reduce_nodes(orc, [bytes(x) for x in nodes])
    return r, ok, "sampled: level-%d blocks %s rebuilt + levels above" % (b, picks)


def corrupt_hook(vals, who):
    """Test-only (MH_BENCH_CORRUPT=<rank or device>): flip one value byte of
    that shard after it was generated, so the root check must fail."""
    if os.environ.get("MH_BENCH_CORRUPT", "") == str(who):
        vals[100:101].bitwise_xor_(1)
        return True
    return False


def reduce_nodes(orc, nodes):
    """The levels above a row of inner nodes with htree's pairing rule
    (htree.go:85-110: h = SHA256(0x01 || l || r), an odd last node moves up
    unchanged) -- no leaf hashing."""
    lvl = list(nodes)
    while len(lvl) > 1:
        nxt = [orc.sha256(b"\x01" + lvl[i] + lvl[i + 1]) for i in range(0, len(lvl) - 1, 2)]
        if len(lvl) % 2:
            nxt.append(lvl[-1])
        lvl = nxt
    return lvl[0]


def global_expected(orc, shard_roots):
    """Root over the shard roots = the root of the whole tree when every shard
    holds a power-of-two count (SURVEY.md finding 3)."""
    return reduce_nodes(orc, shard_roots)


def cgroup_cpus():
    """CPU quota of this process's cgroup (cpu.max), or None if unlimited /
    unreadable: the box's CPU share can be far below what affinity shows."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(seconds):
    """Oracle (C restatement, oracle/) on the host, SHA-NI if present: one thread
    (the Go reference builds a tx's tree in one goroutine), every host thread
    this process may use (sched_getaffinity, SURVEY 8(d) "all cores") and 16
    threads (the GPU box's CPU share), splitting the leaves into power-of-two
    chunks as the GPU path does."""
    orc = _oracle()

    def run(n, threads, reps=5):
        """1 warm-up, then the median of `reps` timed builds."""
        vals = orc.fill_random(n * VAL_LEN, 2).reshape(n, VAL_LEN)
        keys = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).reshape(n, KEY_LEN)
        orc.build_entries_fixed(1, keys, vals, nthreads=threads)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            orc.build_entries_fixed(1, keys, vals, nthreads=threads)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    probe = 1 << 13
    dt = run(probe, 1, reps=1)
    # single thread: the largest power-of-two prefix that fits the time budget
    # (whole 2^20 workload takes ~0.7 s with SHA-NI, so normally all of it)
    n = int(min(N_ENTRIES, max(probe, probe * seconds / 6 / max(dt, 1e-6))))
    n = 1 << (n.bit_length() - 1)
    dt1 = run(n, 1)
    avail = host_threads()
    dta = run(N_ENTRIES, avail)
    t16 = min(16, avail)
    dt16 = dta if t16 == avail else run(N_ENTRIES, t16)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    gib = lambda t: round(N_ENTRIES * VAL_LEN / t / 2 ** 30, 4)  # noqa: E731
    return {
        "value": gib(dta),
        "unit": "GiB/s",
        "cores": avail,
        "cores_available": avail,
        "cgroup_cpu_quota": cgroup_cpus(),
        "cpu_model": model,
        "kind": "port",
        "sample": "htree build over all 2^20 x 1 KiB entries (key BE64(i), v1, seed 2), %d "
                  "threads (every CPU in this process's affinity mask) over power-of-two leaf "
                  "chunks, median of 5 = %.3f s; SHA-NI=%s; CPU: %s"
                  % (avail, dta, orc.has_shani(), model),
        "threads_16": {"value": gib(dt16), "unit": "GiB/s", "cores": t16,
                       "sample": "same build on %d threads (the GPU box's CPU share), median of "
                                 "5 = %.3f s" % (t16, dt16)},
        "single_thread": {"value": round(n * VAL_LEN / dt1 / 2 ** 30, 4), "unit": "GiB/s",
                          "cores": 1, "sample": "first %d entries, median of 5 = %.2f s" % (n, dt1)},
    }


def secondary_config(a):
    """--config c3 / c5 on one GPU: the bench_workloads.py measurement in this
    file's JSON contract, with the oracle timed beside it (cpu_baseline)."""
    import torch  # noqa: F401
    import bench_workloads as bw
    wa = bw.make_parser().parse_args(["--workload", a.config, "--steps", str(a.steps),
                                      "--warmup", str(a.warmup)])
    r = bw.run_single(wa)
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle as orc
    orc.use_shani(True)
    if a.config == "c3":
        M, t = 10 ** 7, r["ms_per_step"] * 1e-3
        alg = 32 * M + 32 * r["dlog_digests"]  # payloads read + dLog written
        ks = r["kernel_ms"]
        out = {"metric": "ahtree batch append, 10^7 x 32 B tx-hash payloads (configs[2])",
               "value": r["value"], "unit": r["unit"], "higher_is_better": True,
               "config": {"workload": "embedded/ahtree batch append of 10^7 payloads to an empty "
                                      "tree, full dLog (124,434,624 digests) in HBM",
                          "appends": M},
               "roofline": {"bound": "hbm", "achieved": round(alg / t / 1e9, 2),
                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                            "kernel": "k_aht_leaves + k_aht_perfect + k_aht_spine_pairs",
                            "kernel_ms": ks,
                            "sha": {"gcomp_per_s": r["gcomp_per_s"],
                                    "peak_gcomp_per_s": SHA_PEAK_GCOMPS,
                                    "frac": round(r["gcomp_per_s"] / SHA_PEAK_GCOMPS, 4)}}}
        # CPU: the oracle's batch append over the first 2^20 payloads (same stream)
        n = 1 << 20
        pay = orc.fill_random(32 * n, 3).reshape(n, 32)
        best = None
        for _ in range(3):
            tr = orc.AHtree(n)
            t0 = time.perf_counter()
            tr.append_batch(pay)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        cpu = {"value": round(n / best / 1e6, 3), "unit": "M appends/s", "cores": 1,
               "kind": "port", "sample": "oracle ahtree batch append of the first 2^20 payloads, "
                                         "single thread, SHA-NI=%s, best of 3 = %.3f s" % (
                                             orc.has_shani(), best)}
    else:
        P, D = 10 ** 6, 24
        t = r["kernel_ms"] * 1e-3
        alg = P * (D * 32 + 32 + 32 + 24)
        out = {"metric": "htree inclusion-proof re-hash, 10^6 proofs x depth 24 (configs[4])",
               "value": r["value"], "unit": r["unit"], "higher_is_better": True,
               "config": {"workload": "htree.VerifyInclusion of 10^6 depth-24 proofs over a "
                                      "2^24-leaf tree, 10 % tampered, bitmap checked",
                          "proofs": P, "depth": D, "bitmap_exact": r["bitmap_exact"]},
               "roofline": {"bound": "hbm", "achieved": round(alg / t / 1e9, 2),
                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                            "kernel": "k_htree_verify", "kernel_ms": r["kernel_ms"],
                            "sha": {"gcomp_per_s": r["gcomp_per_s"],
                                    "peak_gcomp_per_s": SHA_PEAK_GCOMPS,
                                    "frac": round(r["gcomp_per_s"] / SHA_PEAK_GCOMPS, 4)}},
               "proof_generation": r.get("proof_generation")}
        # CPU: the oracle's VerifyInclusion over 2^17 proofs of a 2^24-leaf tree
        # whose levels come from the device build of the same digests
        import immustore_amd as m
        from immustore_amd import _native as N
        W, n = 1 << D, 1 << 17
        dig = torch.empty(W * 32, dtype=torch.uint8, device="cuda")
        ctx = m.Context(0)
        L = N.load()
        N.check(L.mh_dev_fill_random(ctx.handle, dig.data_ptr(), dig.numel(), 5))
        lv = torch.empty(m.levels_len(W) * 32, dtype=torch.uint8, device="cuda")
        rt = torch.empty(32, dtype=torch.uint8, device="cuda")
        N.check(L.mh_dev_htree_build_digests(ctx.handle, dig.data_ptr(), W, lv.data_ptr(),
                                             rt.data_ptr()))
        torch.cuda.synchronize()
        levels = lv.cpu().numpy().reshape(-1, 32)
        digs = dig.cpu().numpy().reshape(-1, 32)
        root = rt.cpu().numpy().tobytes()
        ctx.close()
        rng = np.random.default_rng(5)
        leaf = rng.integers(0, W, n, dtype=np.int64)
        offs = np.array([m.level_offset(W, l) for l in range(D)], np.int64)
        terms = levels[offs[None, :] + ((leaf[:, None] >> np.arange(D)[None, :]) ^ 1)]
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            c, _ = orc.htree_verify_batch(leaf.astype(np.uint64), W, terms, digs[leaf], root)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        assert c == n
        cpu = {"value": round(n / best / 1e6, 3), "unit": "M proofs/s", "cores": 1,
               "kind": "port", "sample": "oracle VerifyInclusion of 2^17 depth-24 proofs, single "
                                         "thread, SHA-NI=%s, best of 3 = %.3f s" % (
                                             orc.has_shani(), best)}
    out.update({"n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": r["ms_per_step"], "scaling": "weak", "vs_baseline": None,
                "dtype": "u32", "data": "synthetic (splitmix64, generated in HBM)",
                "cpu_baseline": None if a.no_cpu_baseline else cpu})
    print(json.dumps(out), flush=True)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch_ranks(a):
    """--gpus N > 1 without a launcher (WORLD_SIZE unset): start N ranks under
    torch.distributed.run as a CHILD process -- before this process touches the
    GPU -- and exit with its status.  Never runs N > 1 as one silent rank."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(a.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def launch_check(a):
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    if world != a.gpus:
        raise SystemExit("process group has %d ranks, --gpus %d" % (world, a.gpus))
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world,
                          "process_group": {"backend": "gloo" if world > 1 else None,
                                            "world_size": world}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cabi_main(a):
    """--api cabi: one process drives devices 0..N-1 through the C ABI
    (mh_multi_create: a context per device + the library's RCCL clique, what
    a cgo caller gets), one mh_multi_dev_htree_build_entries_fixed per step:
    per-device subtree over its resident entries, RCCL all-gather of the N
    subtree roots, the top levels on every device.  --inflight D cliques over
    the same devices, each driven by its own host thread (a clique has one
    stream per device and one build at a time): D builds in flight, as D
    concurrent committers of a Go process would have them."""
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        raise SystemExit("--api cabi is one process: run it without torch.distributed.run")
    import torch
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if ndev < a.gpus:
        raise SystemExit("--api cabi --gpus %d: only %d device(s) visible" % (a.gpus, ndev))
    import immustore_amd as m
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    L = N.load()
    K = a.gpus
    VAL = 4096 if a.config == "c4" else VAL_LEN
    n = a.entries or ((1 << 23) if a.config == "c4" else N_ENTRIES)
    D = max(1, a.inflight if a.inflight is not None else 2)
    mds = [MultiDevice(list(range(K))) for _ in range(D)]
    md = mds[0]
    devs = [torch.device("cuda", d) for d in range(K)]
    vals = [torch.empty(n * VAL, dtype=torch.uint8, device=d) for d in devs]
    keys = [torch.empty(n * KEY_LEN, dtype=torch.uint8, device=d) for d in devs]
    for d in range(K):
        torch.cuda.synchronize(devs[d])
        N.check(L.mh_dev_fill_random(md.ctx_handle(d), vals[d].data_ptr(), vals[d].numel(), 2 + d))
        N.check(L.mh_dev_fill_keys_be64(md.ctx_handle(d), keys[d].data_ptr(), n, d * n))
    md.synchronize()
    corrupted = [d for d in range(K) if corrupt_hook(vals[d], d)]
    for d in devs:
        torch.cuda.synchronize(d)
    # outputs per clique (the builds in flight write concurrently); inputs shared
    lvs = [[torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device=d) for d in devs]
           for _ in range(D)]
    tops = [[torch.empty(max(m.levels_len(K), 1) * 32, dtype=torch.uint8, device=d) for d in devs]
            for _ in range(D)]
    rts = [[torch.empty(32, dtype=torch.uint8, device=d) for d in devs] for _ in range(D)]
    lv, rt = lvs[0], rts[0]
    for d in devs:
        torch.cuda.synchronize(d)
    ptr = lambda ts: [t.data_ptr() for t in ts]  # noqa: E731
    pk, pv = ptr(keys), ptr(vals)
    outs = [(ptr(lvs[j]), ptr(tops[j]), ptr(rts[j])) for j in range(D)]

    def step(j=0):
        pl, pt, pr = outs[j]
        mds[j].dev_build_entries_fixed(1, n, pk, KEY_LEN, pv, VAL, pl, pt, pr)

    def run_steps(total):
        """total builds over the D cliques, one host thread each (ctypes
        releases the GIL inside the call), then every clique synchronised"""
        import threading
        th = [threading.Thread(target=lambda j=j: [step(j) for _ in range(j, total, D)])
              for j in range(1, D)]
        for t in th:
            t.start()
        for _ in range(0, total, D):
            step(0)
        for t in th:
            t.join()
        for x in mds:
            x.synchronize()

    pre = 0
    if a.prewarm > 0:
        tp = time.perf_counter()
        while time.perf_counter() - tp < a.prewarm:
            run_steps(8 * D)
            pre += 8 * D
    run_steps(a.warmup)
    c0 = md.ctx_handle(0)
    t0 = time.perf_counter()
    run_steps(a.steps)
    elapsed = time.perf_counter() - t0
    # device 0's kernel time from a pass after the timed region (the timing
    # events stay out of it)
    N.check(L.mh_ctx_timing_reset(c0))
    N.check(L.mh_ctx_set_timing(c0, 1))
    for _ in range(min(a.steps, 50)):
        step()
    md.synchronize()
    N.check(L.mh_ctx_set_timing(c0, 0))
    import ctypes as C
    ms, cnt = C.c_double(), C.c_uint64()
    N.check(L.mh_ctx_timing(c0, b"entries_fixed", C.byref(ms), C.byref(cnt)))
    kern_ms = ms.value / max(cnt.value, 1)
    # the root check: every device's subtree (top of its levels) vs the
    # oracle's rebuild of its shard, every device's global root vs the
    # oracle's root over those (after the timed region)
    tc = time.perf_counter()
    orc = _oracle()
    threads = host_threads()
    depth = (n - 1).bit_length()
    o_subs, blocks_ok, sub_ok, mode = [], True, True, None
    for d in range(K):
        r, bo, mode = oracle_shard_root(orc, n, VAL, 2 + d, d * n, lv[d], threads)
        o_subs.append(r)
        blocks_ok &= bo
        top_off = m.level_offset(n, depth)
        sub_ok &= lv[d][top_off * 32:(top_off + 1) * 32].cpu().numpy().tobytes() == r
    want = global_expected(orc, o_subs)
    glob_ok = all(r.cpu().numpy().tobytes() == want for rr in rts for r in rr)  # every clique
    exact = K == 1 or (n & (n - 1)) == 0
    rcheck = {"vs": "oracle", "ok": bool(exact and blocks_ok and sub_ok and glob_ok),
              "n": K * n, "shards": K, "mode": mode, "root": want.hex(),
              "subtree_roots_ok": bool(sub_ok), "global_roots_ok": bool(glob_ok),
              "host_threads": threads, "corrupted_shards": corrupted,
              "seconds": round(time.perf_counter() - tc, 2)}
    lpl = int(os.environ.get("MH_LPL", "2" if n >= 2 * 262144 else "1"))
    wgl = int(os.environ.get("MH_WG_LEVELS", "1"))
    ltop = min({1: 0, 2: 1, 4: 2}[lpl] + wgl, (n - 1).bit_length())
    alg_bytes = n * (VAL + KEY_LEN) + 32 * sum(-(-n // (1 << l)) for l in range(ltop + 1))
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    step_achieved = alg_bytes / (elapsed / a.steps) / 1e9
    out = {
        "metric": "device-resident GiB/s hashed, htree build, 1M x 1KiB leaves" if a.config == "c2"
        else "device-resident GiB/s hashed, htree build, 2^23 x 4KiB leaves per GPU (configs[3])",
        "value": round(K * n * VAL / elapsed * a.steps / 2 ** 30, 3),
        "unit": "GiB/s", "n_gpus": K, "api": "cabi", "rccl_ranks": K if md.uses_rccl() else 0,
        "process_group": None, "steps": a.steps, "warmup": a.warmup,
        "clock_prewarm": {"seconds": a.prewarm, "builds": pre},
        "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (splitmix64 values generated in HBM, keys BE64(i))",
        "config": {"workload": "htree build over %d x %d B entries per device, %d devices, "
                               "one process (mh_multi_dev_htree_build_entries_fixed)" % (n, VAL, K),
                   "entries_per_gpu": n, "value_len": VAL, "key_len": KEY_LEN,
                   "parallelism": "subtree shard per device + in-library RCCL all-gather of "
                                  "roots" if K > 1 else "single device (RCCL clique of 1)",
                   "builds_in_flight": D},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "k_entries_fixed", "kernel_ms": round(kern_ms, 4),
                     "kernel_ms_source": "device 0's launches in a pass after the timed region "
                                         "(clique 0 alone, one build at a time: not contended)",
                     "alg_bytes_per_launch": alg_bytes,
                     "per_step": {"achieved": round(step_achieved, 2),
                                  "frac": round(step_achieved / HBM_PEAK_GBS, 4)}},
        "cpu_baseline": None,
        "root_check": rcheck,
    }
    print(json.dumps(out), flush=True)
    for x in mds:
        x.close()
    if not rcheck["ok"]:
        print("root_check FAILED: %s" % json.dumps(rcheck), file=sys.stderr, flush=True)
        raise SystemExit(1)


def root_check_ranks(a, n, val, rank, world, dist, backend, dev, levels_dev, sub_root_dev,
                     glob_root_dev, corrupted, seed=None):
    """Every rank rebuilds its own shard with the oracle on its share of the
    host cores; the 128-byte records (device subtree root, device global
    root, oracle shard root, block verdict) are all-gathered and rank 0
    compares every device root with the oracle's whole-tree root; the verdict
    is shared so every rank exits with the same status."""
    import torch
    t0 = time.perf_counter()
    orc = _oracle()
    threads = host_threads(int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    o_sub, blocks_ok, mode = oracle_shard_root(orc, n, val, 2 + rank if seed is None else seed,
                                               rank * n, levels_dev, threads)
    rec = np.zeros(128, np.uint8)
    rec[0:32] = sub_root_dev.cpu().numpy()
    rec[32:64] = glob_root_dev.cpu().numpy()
    rec[64:96] = np.frombuffer(o_sub, np.uint8)
    rec[96] = int(blocks_ok)
    rec[97] = int(corrupted)
    if dist:
        on = torch.device("cpu") if backend == "gloo" else dev
        g = torch.empty(world * 128, dtype=torch.uint8, device=on)
        dist.all_gather_into_tensor(g, torch.from_numpy(rec).to(on))
        recs = g.cpu().numpy().reshape(world, 128)
    else:
        recs = rec.reshape(1, 128)
    exact = world == 1 or (n & (n - 1)) == 0  # top levels exact for power-of-two shards
    want = global_expected(orc, [recs[r, 64:96].tobytes() for r in range(world)])
    ok = exact and all(recs[r, 96] == 1 for r in range(world)) and \
        all(recs[r, 0:32].tobytes() == recs[r, 64:96].tobytes() for r in range(world)) and \
        all(recs[r, 32:64].tobytes() == want for r in range(world))
    if dist:
        f = torch.tensor([int(ok)], dtype=torch.int64,
                         device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(f.item())
    return {"vs": "oracle", "ok": bool(ok), "n": world * n, "shards": world, "mode": mode,
            "root": want.hex(), "host_threads_per_rank": threads,
            "corrupted_shards": [r for r in range(world) if recs[r, 97]],
            "seconds": round(time.perf_counter() - t0, 2),
            "what": "each rank's subtree root and global root vs the oracle's rebuild of the "
                    "same splitmix64 values / BE64 keys (embedded/htree/htree.go:68-113); "
                    "after the timed region"}


def cabi_c3(a):
    """--api cabi --config c3: syncBinaryLinking's replay (immustore.go:
    1198-1232, reached from :686-693) the way a Go process drives the node's
    GPUs: mh_multi_dev_ahtree_append_batch of `total` payloads (default 10^7
    x 32 B, BASELINE configs[2]) onto a tree of n0 = 10^6 + 3 whose peaks
    were read back with mh_dev_ahtree_peaks, cut into ranges over devices
    0..N-1 (one RCCL clique), each device keeping only its range's digests.
    One step = the whole batch appended again onto the same old tree.  After
    the timed region: RootAt(n0 + total) and sampled digests / roots of every
    range vs the oracle's append of all n0 + total payloads."""
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        raise SystemExit("--api cabi is one process: run it without torch.distributed.run")
    import torch
    K = a.gpus
    if torch.cuda.device_count() < K:
        raise SystemExit("--api cabi --gpus %d: only %d device(s) visible"
                         % (K, torch.cuda.device_count()))
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice, ahtree_range_plan
    L = N.load()
    up = L.mh_ahtree_nodes_upto
    n0, total, plen, seed = a.n0, a.entries or 10 ** 7, 32, 3
    md = MultiDevice(list(range(K)))
    devs = [torch.device("cuda", d) for d in range(K)]
    # the old tree: its n0 appends on device 0, only its peaks kept
    c0 = md.ctx_handle(0)
    pk = np.zeros(32 * bin(n0).count("1"), np.uint8)
    if n0:
        p0 = torch.empty(n0 * plen, dtype=torch.uint8, device=devs[0])
        d0 = torch.empty(up(n0) * 32, dtype=torch.uint8, device=devs[0])
        torch.cuda.synchronize(devs[0])
        N.check(L.mh_dev_fill_random(c0, p0.data_ptr(), p0.numel(), seed))
        N.check(L.mh_dev_ahtree_append_batch(c0, d0.data_ptr(), 0, p0.data_ptr(), n0, plen, None))
        N.check(L.mh_dev_ahtree_peaks(c0, d0.data_ptr(), n0, pk.ctypes.data))
        md.synchronize()
        del p0, d0
    shard_bits, b = ahtree_range_plan(n0, total, K)
    G = len(b) - 1
    # range d = appends (b[d], b[d+1]]: payloads b[d] .. b[d+1]-1 of the one
    # splitmix64 stream (word offset 4 b[d])
    pay, dl, ro = [None] * K, [None] * K, [None] * K
    for d in range(G):
        cnt = b[d + 1] - b[d]
        pay[d] = torch.empty(cnt * plen, dtype=torch.uint8, device=devs[d])
        dl[d] = torch.empty((up(b[d + 1]) - up(b[d])) * 32, dtype=torch.uint8, device=devs[d])
        ro[d] = torch.empty(cnt * 32, dtype=torch.uint8, device=devs[d])
        torch.cuda.synchronize(devs[d])
        sd = (seed + b[d] * (plen // 8) * SPLITMIX_G) & 0xFFFFFFFFFFFFFFFF
        N.check(L.mh_dev_fill_random(md.ctx_handle(d), pay[d].data_ptr(), pay[d].numel(), sd))
    md.synchronize()
    corrupted = [d for d in range(G) if corrupt_hook(pay[d], d)]
    for d in devs:
        torch.cuda.synchronize(d)
    ptr = lambda ts: [t.data_ptr() if t is not None else None for t in ts]  # noqa: E731
    pp, pd, pr = ptr(pay), ptr(dl), ptr(ro)
    pkb = pk.tobytes() if n0 else None

    def step():
        md.dev_ahtree_append_batch(total, pp, plen, pd, pr, n0=n0, peaks=pkb)

    pre = 0
    if a.prewarm > 0:
        tp = time.perf_counter()
        while time.perf_counter() - tp < a.prewarm:
            for _ in range(4):
                step()
                pre += 1
            md.synchronize()
    for _ in range(a.warmup):
        step()
    md.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    md.synchronize()
    elapsed = time.perf_counter() - t0
    ms = elapsed / a.steps * 1e3
    # device 0's kernels in a pass after the timed region
    N.check(L.mh_ctx_timing_reset(c0))
    N.check(L.mh_ctx_set_timing(c0, 1))
    kp = min(a.steps, 10)
    for _ in range(kp):
        step()
    md.synchronize()
    N.check(L.mh_ctx_set_timing(c0, 0))
    import ctypes as C
    kms = {}
    for k in ("aht_leaves", "aht_perfect", "aht_spine", "aht_top", "aht_gather"):
        t, c = C.c_double(), C.c_uint64()
        N.check(L.mh_ctx_timing(c0, k.encode(), C.byref(t), C.byref(c)))
        if c.value:
            kms[k] = round(t.value / kp, 3)
    # ---- check vs the oracle's append of every payload
    tc = time.perf_counter()
    orc = _oracle()
    allp = orc.fill_random((n0 + total) * plen, seed).reshape(n0 + total, plen)
    o = orc.AHtree(n0 + total)
    o.append_batch(allp)
    ref = o.dlog  # (>= nodesUpto(n0 + total), 32), no copy
    ok = True
    rng = np.random.default_rng(7)
    for d in range(G):
        g = dl[d].view(-1, 32)
        nd = g.shape[0]
        idx = np.unique(np.concatenate([np.arange(min(nd, 512)), np.arange(max(nd - 512, 0), nd),
                                        rng.integers(0, nd, 2048)]))
        got = g[torch.from_numpy(idx).to(g.device)].cpu().numpy()
        ok &= bool(np.array_equal(got, ref[up(b[d]) + idx]))
        r = ro[d].view(-1, 32)
        cnt = b[d + 1] - b[d]
        for j in sorted({0, cnt // 2, cnt - 1, int(rng.integers(0, cnt))}):
            ok &= r[j].cpu().numpy().tobytes() == bytes(o.root_at(b[d] + j + 1)[1])
    want = bytes(o.root_at(n0 + total)[1])
    last = ro[G - 1].view(-1, 32)[-1].cpu().numpy().tobytes()
    ok &= last == want
    rcheck = {"vs": "oracle", "ok": bool(ok), "n": n0 + total, "root": want.hex(),
              "what": "RootAt(n0 + total) and, per range, its first / last 512 and 2048 random "
                      "digests and 4 RootAt values vs orc.AHtree over all n0 + total payloads "
                      "(embedded/ahtree/ahtree.go:246-373, 727-771)",
              "corrupted_ranges": corrupted, "seconds": round(time.perf_counter() - tc, 2)}
    new_digests = up(n0 + total) - up(n0)
    alg = total * plen + 32 * new_digests
    out = {"metric": "ahtree replay append (syncBinaryLinking), %d x %d B payloads onto a tree of "
                     "%d, through the C ABI across %d device(s)" % (total, plen, n0, K),
           "value": round(total / elapsed * a.steps / 1e6, 3), "unit": "M appends/s",
           "n_gpus": K, "api": "cabi", "rccl_ranks": K if (md.uses_rccl() and G > 1) else 0,
           "steps": a.steps, "warmup": a.warmup,
           "clock_prewarm": {"seconds": a.prewarm, "appends_batches": pre},
           "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (splitmix64 payloads generated in HBM)",
           "config": {"workload": "mh_multi_dev_ahtree_append_batch onto old peaks from "
                                  "mh_dev_ahtree_peaks", "n0": n0, "appends": total,
                      "payload_len": plen, "ranges": G, "range_bounds": b,
                      "shard_bits": shard_bits,
                      "dlog_bytes_per_device": [int(t.numel()) if t is not None else 0
                                                for t in dl]},
           "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": None, "alg_bytes_per_step": alg,
                        "note": "payloads read + new dLog digests written, whole job per step",
                        "kernel_ms_device0": kms,
                        "sha": {"gcomp_per_s": round((total + 2 * (new_digests - total)) /
                                                     (ms * 1e-3) / 1e9, 2),
                                "peak_gcomp_per_s": SHA_PEAK_GCOMPS}},
           "cpu_baseline": None, "root_check": rcheck}
    print(json.dumps(out), flush=True)
    md.close()
    if not ok:
        print("root_check FAILED: %s" % json.dumps(rcheck), file=sys.stderr, flush=True)
        raise SystemExit(1)


def cabi_txlog(a):
    """--api cabi --config txlog: SURVEY.md 8(a) a14 / 8(f) row 2, the read
    path's re-hash of a tx log (tx.go:388-630; the replay of
    immustore.go:1198-1223 and the indexer's readTx, indexer.go:570) the way a
    Go process drives the node's GPUs: mh_multi_txlog_validate over devices
    0..N-1 -- the log (2^16 records x 16 entries, 75.5 MB, pinned as the cgo
    shim's arena) cut at record boundaries, every part copied over its own
    PCIe link and validated on its device.  After the timed region every Alh
    and status is checked against the oracle's (oracle/, which also sealed the
    log); MH_BENCH_CORRUPT=0 flips one stored hVal so the check must fail."""
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        raise SystemExit("--api cabi is one process: run it without torch.distributed.run")
    import torch
    K = a.gpus
    if torch.cuda.device_count() < K:
        raise SystemExit("--api cabi --gpus %d: only %d device(s) visible"
                         % (K, torch.cuda.device_count()))
    import bench_workloads as bw
    from immustore_amd.multi import MultiDevice
    from immustore_amd.txlayer import TX_HEADER
    orc = _oracle()
    ntx, ne, kl = a.entries or (1 << 16), 16, 16
    buf = bw.txlog_records(ntx, ne, kl)
    rec = buf.shape[1]
    _, n, _, alh_o, _ = orc.txlog_validate(buf.reshape(-1))  # sealed by the oracle
    assert n == ntx
    buf[:, rec - 32:] = alh_o
    corrupted = os.environ.get("MH_BENCH_CORRUPT", "") == "0"
    if corrupted:
        buf[ntx // 2, rec - 33] ^= 1  # the last entry's hVal of the middle record
    pin = torch.empty(buf.size, dtype=torch.uint8).pin_memory()
    raw = pin.numpy()
    raw[:] = buf.reshape(-1)
    outs = (torch.empty(ntx * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy()
            .view(TX_HEADER),
            torch.empty(ntx * 32, dtype=torch.uint8).pin_memory().numpy().reshape(ntx, 32),
            torch.empty(ntx, dtype=torch.int32).pin_memory().numpy())
    md = MultiDevice(list(range(K)))

    def step():
        r = md.txlog_validate(raw, out=outs)
        assert r[0] == 0 and r[1] == ntx

    pre = 0
    tp = time.perf_counter()
    while time.perf_counter() - tp < a.prewarm:
        step()
        pre += 1
    for _ in range(a.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    elapsed = time.perf_counter() - t0
    ms = elapsed / a.steps * 1e3
    # ---- check vs the oracle (the log's own stored Alh values, recomputed)
    tc = time.perf_counter()
    r = md.txlog_validate(raw, out=outs)
    o = orc.txlog_validate(raw)
    ok = r[:3] == (o[0], o[1], o[2]) and bool(np.array_equal(r[4], o[3])) and \
        list(r[5]) == list(o[4]) and not r[5].any()
    rcheck = {"vs": "oracle", "ok": bool(ok), "records": ntx,
              "bad_records": [int(x) for x in np.nonzero(r[5])[0][:8]],
              "what": "every record's recomputed Alh and per-tx status vs orc.txlog_validate "
                      "(tx.go:388-630) over the same log, all valid",
              "corrupted": corrupted, "seconds": round(time.perf_counter() - tc, 2)}
    md.close()
    out = {"metric": "tx-log read-path validation (a14), %d records x %d entries, through the C "
                     "ABI across %d device(s)" % (ntx, ne, K),
           "value": round(ntx / (ms * 1e-3) / 1e6, 3), "unit": "M tx/s", "n_gpus": K, "api": "cabi",
           "steps": a.steps, "warmup": a.warmup, "clock_prewarm": {"seconds": a.prewarm,
                                                                   "calls": pre},
           "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "u32",
           "data": "synthetic v1 records (bench_workloads.txlog_records), sealed by the oracle, "
                   "pinned host log and outputs",
           "config": {"workload": "mh_multi_txlog_validate: the log cut at record boundaries, "
                                  "one part per device over its own PCIe link",
                      "log_bytes": int(raw.size), "records": ntx, "entries_per_record": ne},
           "log_GBps_incl_parse_and_h2d": round(raw.size / (ms * 1e-3) / 1e9, 2),
           "cpu_baseline": None, "root_check": rcheck}
    print(json.dumps(out), flush=True)
    if not ok:
        print("root_check FAILED: %s" % json.dumps(rcheck), file=sys.stderr, flush=True)
        raise SystemExit(1)


def main():
    a = parse()
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if a.api == "cabi":
        if a.config == "txlog":
            return cabi_txlog(a)
        return cabi_c3(a) if a.config == "c3" else cabi_main(a)
    if a.config == "txlog":
        raise SystemExit("--config txlog runs through --api cabi (one process over N devices); "
                         "one GPU: bench_workloads.py --workload txlog")
    # MH_DIST_FORCE_PG=1: the --gpus N code path (process group, comm stream,
    # all-gather of the roots over RCCL, the top levels, the root-check
    # records) even at N = 1, launched as one torch.distributed.run rank
    force_pg = os.environ.get("MH_DIST_FORCE_PG", "") == "1"
    if (a.gpus > 1 or force_pg) and "WORLD_SIZE" not in os.environ:
        raise SystemExit(relaunch_ranks(a))
    if a.launch_check:
        return launch_check(a)
    if a.config in ("c3", "c5"):
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise SystemExit("--config c3/c5 here is one GPU; multi-GPU: bench_workloads.py "
                             "under torch.distributed.run")
        return secondary_config(a)
    import torch
    import immustore_amd as m
    from immustore_amd import _native as N
    from immustore_amd import sharding

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (a.gpus, world))
    strong = a.scaling == "strong"
    if strong and (a.config != "c2" or world & (world - 1)):
        raise SystemExit("--scaling strong: --config c2 and a power-of-two --gpus")
    dist = None
    # one process per GPU; MH_DIST_BACKEND=gloo rehearses several ranks on
    # fewer GPUs (device = local rank modulo the visible devices)
    backend = os.environ.get("MH_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend != "gloo" and world > 1 and local >= ndev:
        raise SystemExit("rank %d has no GPU (%d visible)" % (local, ndev))
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    local = dev.index
    if world > 1 or force_pg:
        import torch.distributed as dist
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != a.gpus:
            raise SystemExit("process group has %d ranks, --gpus %d"
                             % (dist.get_world_size(), a.gpus))

    # D builds in flight (--inflight), each on its own HIP stream with its own
    # level buffers: the latency-bound top of one tree overlaps the leaf
    # hashing of the next, as concurrent commits do in immudb (up to
    # MaxConcurrency precommits, embedded/store/options.go:35).  D = 1 is
    # strictly sequential.
    D = max(1, a.inflight if a.inflight is not None else 3)
    # With a process group the build streams are high-priority streams: HIP
    # gives those a hardware-queue pool of their own, so the three builds keep
    # three queues next to the process group's streams (with the normal pool of
    # GPU_MAX_HW_QUEUES = 4 two builds shared one queue and ran back to back:
    # one nccl rank 1154 -> 1264 GiB/s, >= 2 leaf kernels running 4 -> 85 % of
    # the time, profiles/pgprof_r05.txt).  MH_BENCH_STREAM_PRIO overrides.
    prio = int(os.environ.get("MH_BENCH_STREAM_PRIO", "-1" if dist else "0"))
    streams = [torch.cuda.current_stream(dev)] if D == 1 else \
        [torch.cuda.Stream(dev, priority=prio) for _ in range(D)]
    ctxs = [m.Context(local, s.cuda_stream) for s in streams]
    ctx = ctxs[0]
    L = N.load()
    VAL = 4096 if a.config == "c4" else VAL_LEN
    n = a.entries or ((1 << 23) if a.config == "c4" else N_ENTRIES)
    if strong:  # one tree of n entries: this rank's aligned 1 / world of it
        if n % world:
            raise SystemExit("--scaling strong: %d entries do not split over %d GPUs" % (n, world))
        n //= world
    seed = shard_seed(rank, n, VAL, strong)
    # inputs resident in HBM before the timed region (synthetic, deterministic)
    vals = torch.empty(n * VAL, dtype=torch.uint8, device=dev)
    keys = torch.empty(n * KEY_LEN, dtype=torch.uint8, device=dev)
    with torch.cuda.stream(streams[0]):
        N.check(L.mh_dev_fill_random(ctx.handle, vals.data_ptr(), vals.numel(), seed))
        N.check(L.mh_dev_fill_keys_be64(ctx.handle, keys.data_ptr(), n, rank * n))
        corrupted = corrupt_hook(vals, rank)
    torch.cuda.synchronize(dev)
    nlv = m.levels_len(n)
    levels = [torch.empty(nlv * 32, dtype=torch.uint8, device=dev) for _ in range(D)]
    root = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(D)]
    top_levels = [torch.empty(max(m.levels_len(world), 1) * 32, dtype=torch.uint8, device=dev)
                  for _ in range(D)]
    groot = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(D)]

    # the all-gather + top levels of build j run on build j's own stream:
    # torch issues every collective of the process group on its one internal
    # stream in host order, so all ranks run their RCCL kernels in the same
    # order without a stream of ours.  A separate comm stream (the round-4
    # form, MH_BENCH_COMM_STREAM=1) costs a HIP hardware queue: with 4 per
    # process (GPU_MAX_HW_QUEUES) three build streams, the PG's stream and a
    # comm stream share them, so two builds end up in one queue and stop
    # overlapping (profiles/pgprof_r05.txt: 1132 vs 1298 GiB/s as one rank).
    sep_comm = dist is not None and D > 1 and os.environ.get("MH_BENCH_COMM_STREAM", "") == "1"
    comm = torch.cuda.Stream(dev) if sep_comm else None
    comm_ctx = m.Context(local, comm.cuda_stream) if sep_comm else None

    def step(k):
        j = k % D
        with torch.cuda.stream(streams[j]):
            N.check(L.mh_dev_htree_build_entries_fixed(ctxs[j].handle, 1, n, keys.data_ptr(),
                                                       KEY_LEN, vals.data_ptr(), VAL, None,
                                                       levels[j].data_ptr(), root[j].data_ptr()))
        if dist:
            # 32 B per rank over RCCL, then the top log2(world) levels locally
            # (immustore_amd/sharding.py; exact by SURVEY.md finding 3)
            s_, c_ = (comm, comm_ctx) if sep_comm else (streams[j], ctxs[j])
            if sep_comm:
                comm.wait_stream(streams[j])
            with torch.cuda.stream(s_):
                g = sharding.allgather_roots(root[j], world)
                N.check(L.mh_dev_htree_reduce_nodes(c_.handle, g.data_ptr(), world,
                                                    top_levels[j].data_ptr(), groot[j].data_ptr()))
            if sep_comm:
                streams[j].wait_stream(comm)

    # clock pre-warm: full builds (same inputs, every level recomputed, nothing
    # kept) for a fixed wall time before the W warmup steps -- with the
    # driver's few-step runs the timed region would otherwise sit on the
    # shader-clock ramp of a GPU that was idle a moment earlier.  Every rank
    # decides after the same chunk of 8 builds, so the RCCL calls match.
    pre = 0
    if a.prewarm > 0:
        tp = time.perf_counter()
        while True:
            for _ in range(8):
                step(pre)
                pre += 1
            torch.cuda.synchronize(dev)
            more = time.perf_counter() - tp < a.prewarm
            if dist:
                # every rank takes the same decision after the same chunk
                f = torch.tensor([int(more)], dtype=torch.int64,
                                 device="cpu" if backend == "gloo" else dev)
                dist.all_reduce(f, op=dist.ReduceOp.MAX)
                more = bool(f.item())
            if not more:
                break
    for k in range(a.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # the per-kernel timing events (two per launch) stay off in the timed
    # region: the contended kernel time comes from a pass of its own below
    for c in ctxs:
        c.timing_reset()
        c.set_timing(a.timing_in_region)
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for c in ctxs:
        c.set_timing(False)
    elapsed = t1 - t0
    if not a.timing_in_region:
        # the same steps (every in-flight stream) with the timing events on
        for c in ctxs:
            c.timing_reset()
            c.set_timing(True)
        for k in range(min(a.steps, 60 * D)):
            step(k)
        torch.cuda.synchronize(dev)
        for c in ctxs:
            c.set_timing(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    k_ms0, k_cnt0 = ctxs[0].timing("entries_fixed")
    # isolated launches (outside the timed region): ISO builds back to back on
    # ONE stream (a single BuildWith chain, i.e. --inflight 1), for the
    # dominant kernel's exclusive duration and the single-build rate
    ISO = 10

    def iso_builds(count):
        for k in range(count):
            with torch.cuda.stream(streams[0]):
                N.check(L.mh_dev_htree_build_entries_fixed(ctxs[0].handle, 1, n, keys.data_ptr(),
                                                           KEY_LEN, vals.data_ptr(), VAL, None,
                                                           levels[0].data_ptr(),
                                                           root[0].data_ptr()))
        torch.cuda.synchronize(dev)

    # the single-build rate without timing events, then the same builds with
    # them for the kernel's own duration
    torch.cuda.synchronize(dev)
    ti0 = time.perf_counter()
    iso_builds(5 * ISO)
    single_ms = (time.perf_counter() - ti0) / (5 * ISO) * 1e3
    ctxs[0].timing_reset()
    ctxs[0].set_timing(True)
    iso_builds(ISO)
    ctxs[0].set_timing(False)
    ims, icnt = ctxs[0].timing("entries_fixed")
    iso_ms = ims / max(icnt, 1)
    iso_reduce_ms = ctxs[0].timing("reduce")[0] / ISO
    # every build's root must be the same tree root (same input each step)
    r0 = root[0].cpu()
    assert all(torch.equal(r0, r.cpu()) for r in root), "in-flight builds disagree"
    rcheck = root_check_ranks(a, n, VAL, rank, world, dist, backend, dev, levels[0], root[0],
                              groot[0] if dist else root[0], corrupted, seed)

    k_ms = sum(c.timing("entries_fixed")[0] for c in ctxs[1:]) + k_ms0
    k_cnt = sum(c.timing("entries_fixed")[1] for c in ctxs[1:]) + k_cnt0
    contended_ms = k_ms / max(k_cnt, 1)
    kern_ms = iso_ms
    # mirrors choose_lpl / launch_entries_fixed in htree_kernels.hip
    lpl = int(os.environ.get("MH_LPL", "2" if n >= 2 * 262144 else "1"))
    # levels written by one launch of the dominant kernel: the lanes' groups
    # up to level log2(lpl), then each workgroup's subtree 8 levels higher
    wgl = int(os.environ.get("MH_WG_LEVELS", "1"))  # default of launch_entries_fixed
    top = min({1: 0, 2: 1, 4: 2}[lpl] + wgl, max(m.levels_len(n) and (n - 1).bit_length(), 0))
    widths = [-(-n // (1 << l)) for l in range(top + 1)]
    nodes_written = sum(widths)
    # algorithmic HBM bytes of one launch of the dominant kernel:
    #   read value + key of every entry, write every level node it produces
    alg_bytes = n * (VAL + KEY_LEN) + 32 * nodes_written
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    # compressions: 16 value blocks + digest + leaf per entry (generic),
    # the constant padding block (compress_kw), 2 per inner node
    node_hashes = nodes_written - n
    valu = (n * (VAL // 64 + 2) * OPS_PER_COMP + n * OPS_PER_COMP_KW +
            2 * node_hashes * OPS_PER_COMP) / (kern_ms * 1e-3)
    comp_rate = (n * (VAL // 64 + 3) + 2 * node_hashes) / (kern_ms * 1e-3)
    # every compression of one whole build (all levels: floor(w / 2) node
    # hashes per level, htree.go:85-110) over the measured time of a step
    all_pairs, w = 0, n
    while w > 1:
        all_pairs += w // 2
        w = -(-w // 2)
    step_comp_rate = (n * (VAL // 64 + 3) + 2 * all_pairs) / (elapsed / a.steps)
    traffic = None
    if a.config == "c2" and os.path.exists(a.traffic_file):
        try:
            traffic = json.load(open(a.traffic_file)).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    total_bytes = world * n * VAL
    value = total_bytes / elapsed * a.steps / 2 ** 30
    # the same algorithmic bytes over the measured time of one step (the
    # builds in flight overlap, so this is a sustained rate, not one launch)
    step_achieved = alg_bytes / (elapsed / a.steps) / 1e9
    out = {
        "metric": "device-resident GiB/s hashed, htree build, 1M x 1KiB leaves" if a.config == "c2"
        else "device-resident GiB/s hashed, htree build, 2^23 x 4KiB leaves per GPU (configs[3])",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "process_group": {"backend": backend if dist else None,
                          "world_size": dist.get_world_size() if dist else 1},
        "steps": a.steps,
        "warmup": a.warmup,
        "clock_prewarm": {"seconds": a.prewarm, "builds": pre,
                          "note": "untimed full builds before the warmup steps (GPU clock ramp)"},
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (splitmix64 values generated in HBM, keys BE64(i))",
        "config": {"workload": "htree build (value SHA-256 + TxEntryDigest_v1_2 + leaf + all "
                               "levels), %d x %d B entries per GPU, %d B keys" % (n, VAL, KEY_LEN)
                   + ("; strong scaling: one %d-entry tree over %d GPUs" % (n * world, world)
                      if strong else ""),
                   "entries_per_gpu": n, "entries_total": n * world, "value_len": VAL,
                   "key_len": KEY_LEN,
                   "parallelism": "subtree shard per GPU + %s all-gather of roots"
                   % ("RCCL" if backend != "gloo" else "gloo") if dist else "single GPU", "lanes_per_leaf_group": lpl,
                   "builds_in_flight": D, "wg_subtree_levels": wgl, "stream_priority": prio},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "traffic_source": os.path.relpath(a.traffic_file, HERE) if traffic else None,
                     "kernel": "k_entries_fixed",
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes,
                     "per_step": {"achieved": round(step_achieved, 2),
                                  "frac": round(step_achieved / HBM_PEAK_GBS, 4),
                                  "note": "alg_bytes_per_launch / ms_per_step: the timed "
                                          "region's own clock, beside the isolated-launch "
                                          "achieved / frac"},
                     "valu": {"achieved_tops": round(valu / 1e12, 2),
                              "peak_tops": round(VALU_PEAK_OPS / 1e12, 2),
                              "frac": round(valu / VALU_PEAK_OPS, 4),
                              "peak_source": "measured SHA-256 register loop 30.9 G comp/s "
                                             "(profiles/microbench_r01.txt) x 1388 VALU "
                                             "instructions per compression (profiles/"
                                             "isa_counts_r01.txt): the issue-weighted peak of "
                                             "this instruction mix; achieved counts the "
                                             "constant-schedule blocks at 901"},
                     "sha": {"gcomp_per_s": round(comp_rate / 1e9, 2),
                             "peak_gcomp_per_s": SHA_PEAK_GCOMPS,
                             "frac": round(comp_rate / 1e9 / SHA_PEAK_GCOMPS, 4),
                             "step": {"gcomp_per_s": round(step_comp_rate / 1e9, 2),
                                      "frac": round(step_comp_rate / 1e9 / SHA_PEAK_GCOMPS, 4),
                                      "note": "every compression of one build (leaf kernel "
                                              "and all levels) per ms_per_step; the builds "
                                              "in flight overlap, so this is the GPU's "
                                              "sustained rate on the workload"}},
                     "reduce_ms_per_build": round(iso_reduce_ms, 4),
                     "kernel_ms_source": "isolated launches: %d builds back to back on one "
                                         "stream after the timed region, HIP events around "
                                         "each k_entries_fixed launch (achieved / frac / valu / "
                                         "sha all use this duration)" % ISO,
                     "contended_kernel_ms": round(contended_ms, 4),
                     "contended_note": "mean launch duration in a pass of the timed "
                                       "region's steps after it (timing events off inside it), where "
                                       "%d builds in flight share the GPU and stretch each "
                                       "launch; not the kernel's own time" % D},
        "single_build": {"builds_in_flight": 1, "ms_per_build": round(single_ms, 4),
                         "gib_per_s": round(n * VAL / (single_ms * 1e-3) / 2 ** 30, 2),
                         "note": "one BuildWith at a time (what one Go committer sees), "
                                 "50 builds back to back, no timing events"},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.config == "c2":
        out["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    out["root_check"] = rcheck
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm_ctx is not None:
        comm_ctx.close()
    for c in ctxs:
        c.close()
    if dist:
        dist.destroy_process_group()
    if not rcheck["ok"]:
        print("root_check FAILED: %s" % json.dumps(rcheck), file=sys.stderr, flush=True)
        raise SystemExit(1)


if __name__ == "__main__":
    main()
