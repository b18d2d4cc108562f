#!/usr/bin/env python3
"""mh_txlog_validate on the bench's a14 log (2^16 records x 16 entries, pinned
input and pinned outputs, as bench_workloads --workload txlog's timed step),
30 calls with nothing after the last: run under rocprofv3 --kernel-trace
--memory-copy-trace and read the last call with tools/trace_window.py."""
import os
import struct
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import immustore_amd as m  # noqa: E402
from immustore_amd.txlayer import TX_HEADER  # noqa: E402

ctx = m.Context(0)
rng = np.random.default_rng(14)
ntx, ne, kl = 1 << 16, 16, 16
ent = 2 + 2 + kl + 4 + 8 + 32
hdr = 96
rec = hdr + ne * ent + 32
buf = np.zeros((ntx, rec), np.uint8)
buf[:, 0:8] = np.arange(1, ntx + 1, dtype=">u8").view(np.uint8).reshape(ntx, 8)
buf[:, 24:88] = rng.integers(0, 256, (ntx, 64), dtype=np.uint8)
buf[:, 89] = 1
buf[:, 92:96] = np.frombuffer(struct.pack(">I", ne), np.uint8)
e = buf[:, hdr:hdr + ne * ent].reshape(ntx, ne, ent)
e[:, :, 3] = kl
e[:, :, 4:4 + kl] = rng.integers(0, 256, (ntx, ne, kl), dtype=np.uint8)
e[:, :, 4 + kl + 12:] = rng.integers(0, 256, (ntx, ne, 32), dtype=np.uint8)
rc, n, used, _, alh, _ = m.txlog_validate(buf.reshape(-1), ctx=ctx)
buf[:, rec - 32:] = alh
pin = torch.empty(buf.size, dtype=torch.uint8).pin_memory()
pin.numpy()[:] = buf.reshape(-1)
outs = (torch.empty(ntx * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER),
        torch.empty(ntx * 32, dtype=torch.uint8).pin_memory().numpy().reshape(ntx, 32),
        torch.empty(ntx, dtype=torch.int32).pin_memory().numpy())
o = (None,) + outs[1:] if os.environ.get("TXB_NO_HDRS") else outs
if os.environ.get("TXTL_PAGEABLE"):  # the log from pageable memory (a plain numpy copy)
    pin = torch.from_numpy(pin.numpy().copy())
ts = []
if os.environ.get("TXTL_CLOG"):  # mh_txlog_validate_clog over the pinned log + its cLog
    from immustore_amd.txlayer import txlog_validate_clog
    clog = b"".join(struct.pack(">QI", k * rec, rec) for k in range(ntx))
    for i in range(30):
        t = time.perf_counter()
        r = txlog_validate_clog(pin.numpy(), pin.numel(), clog, ctx=ctx, out=o)
        ts.append(time.perf_counter() - t)
        assert r[0] == 0 and r[1] == 0 and not o[2].any()
for i in range(0 if ts else 30):
    t = time.perf_counter()
    r = m.txlog_validate(pin.numpy(), ctx=ctx, out=o)
    ts.append(time.perf_counter() - t)
    assert r[0] == 0 and r[1] == ntx and not r[5].any()
print("ms per call: last 10 median %.3f min %.3f" % (sorted(ts[-10:])[5] * 1e3, min(ts) * 1e3))
