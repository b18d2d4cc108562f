#!/usr/bin/env python3
"""60 single htree builds (C2: 2^20 x 1 KiB, device resident, one stream, no
timing events) and nothing after: run under rocprofv3 --kernel-trace and read
the last builds with tools/trace_window.py."""
import sys
import time

import torch

sys.path.insert(0, ".")
import immustore_amd as m  # noqa: E402
from immustore_amd import _native as N  # noqa: E402

n, VAL, KL = 1 << 20, 1024, 8
dev = torch.device("cuda", 0)
ctx = m.Context(0, torch.cuda.current_stream(dev).cuda_stream)
L = N.load()
vals = torch.empty(n * VAL, dtype=torch.uint8, device=dev)
keys = torch.empty(n * KL, dtype=torch.uint8, device=dev)
N.check(L.mh_dev_fill_random(ctx.handle, vals.data_ptr(), vals.numel(), 2))
N.check(L.mh_dev_fill_keys_be64(ctx.handle, keys.data_ptr(), n, 0))
levels = torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device=dev)
root = torch.empty(32, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
t = []
for k in range(60):
    t0 = time.perf_counter()
    N.check(L.mh_dev_htree_build_entries_fixed(ctx.handle, 1, n, keys.data_ptr(), KL, vals.data_ptr(),
                                               VAL, None, levels.data_ptr(), root.data_ptr()))
    torch.cuda.synchronize()
    t.append(time.perf_counter() - t0)
print("ms per build (synchronised each): median %.4f min %.4f" % (sorted(t[10:])[25] * 1e3, min(t) * 1e3))
