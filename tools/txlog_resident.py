#!/usr/bin/env python3
"""a14 with the log resident in HBM (mh_txlog_validate_resident): one group,
i.e. ONE launch of the a14 kernel over every record after the host hop -- the
kernel's own time for the scrub / re-validate caller.  Prints one JSON line
with the call time and the kernel time per call (HIP events); MH_TXLOG_KERNEL
picks the kernel, MH_TXLOG_PROBE=1 adds the per-phase stamps on stderr.

    python3 tools/txlog_resident.py [records] [calls]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    import torch
    import immustore_amd as m
    import bench_workloads as bw
    ntx = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    ctx = m.Context(0)
    buf = bw.txlog_records(ntx, 16, 16)
    rec = buf.shape[1]
    raw = buf.reshape(-1)
    _, n, _, _, alh, _ = m.txlog_validate(raw, ctx=ctx)
    buf[:, rec - 32:] = alh
    d = torch.zeros(raw.size + 256, dtype=torch.uint8, device="cuda")
    d[:raw.size].copy_(torch.from_numpy(raw))
    torch.cuda.synchronize()
    kern = os.environ.get("MH_TXLOG_KERNEL", "wave")
    name = {"blk": "txlog_blk", "group": "txlog_group", "lanes": "txlog_lanes"}.get(kern, "txlog_wave")
    for _ in range(20):
        r = m.txlog_validate(raw, ctx=ctx, dev=d.data_ptr())
        assert r[0] == 0 and r[1] == ntx and not r[5].any()
    ctx.timing_reset()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(calls):
        m.txlog_validate(raw, ctx=ctx, dev=d.data_ptr())
    t = (time.perf_counter() - t0) / calls
    ctx.set_timing(False)
    if os.environ.get("MH_TXLOG_FUSED") == "0":  # the six-launch chain: every kernel of the call
        kms = sum(ctx.timing(k)[0] for k in ("tx_hdr_from_raw", "txe_index", "txe_leaf",
                                             "small_roots", "seg_level", "tx_alh"))
        cnt = ctx.timing("txe_leaf")[1]
        kern = "chain"
    else:
        kms, cnt = ctx.timing(name)
    comps = ntx * (16 * 2 + 2 * 15 + 4)
    print(json.dumps({"kernel": kern, "records": ntx, "ms_per_call": round(t * 1e3, 4),
                      "kernel_ms": round(kms / max(cnt, 1), 4),
                      "sha_frac": round(comps / (kms / max(cnt, 1) * 1e-3) / 1e9 / 30.9, 4)}))


if __name__ == "__main__":
    main()
