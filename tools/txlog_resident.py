#!/usr/bin/env python3
"""a14 with the log resident in HBM (mh_txlog_validate_resident): one group,
i.e. ONE launch of the a14 kernel over every record after the host hop -- the
kernel's own time for the scrub / re-validate caller.  Prints one JSON line
with the call time and the kernel time per call (HIP events); MH_TXLOG_KERNEL
picks the kernel (MH_TXLOG_LANES the lanes per record).

    python3 tools/txlog_resident.py [records] [calls] [entries per record]
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
    ne = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    buf = bw.txlog_records(ntx, ne, 16)
    rec = buf.shape[1]
    raw = buf.reshape(-1)
    _, n, _, _, alh, _ = m.txlog_validate(raw, ctx=ctx)
    buf[:, rec - 32:] = alh
    d = torch.zeros(raw.size + 256, dtype=torch.uint8, device="cuda")
    d[:raw.size].copy_(torch.from_numpy(raw))
    torch.cuda.synchronize()
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
    # the kernel the call picked (lanes by default for one group of >= 16384
    # records; MH_TXLOG_KERNEL=wave | lanes forces one)
    kern, (kms, cnt) = max((("lanes", ctx.timing("txlog_lanes")), ("wave", ctx.timing("txlog_wave"))),
                           key=lambda x: x[1][1])
    comps = ntx * (ne * 2 + 2 * (ne - 1) + 4)
    print(json.dumps({"kernel": kern, "records": ntx, "entries": ne, "ms_per_call": round(t * 1e3, 4),
                      "kernel_ms": round(kms / max(cnt, 1), 4),
                      "sha_frac": round(comps / (kms / cnt * 1e-3) / 1e9 / 30.9, 4) if kms else None}))


if __name__ == "__main__":
    main()
