"""A/B of the leaves-from-digests kernel's entries per lane (MH_DIGEST_LPL,
read per build): mh_dev_htree_build_digests over 2^20 and 2^24 device digests,
isolated builds on one stream, HIP-event time of the leaf launch ("leaves")
and of the whole build.  Prints one JSON line per (lpl, n)."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import immustore_amd as m  # noqa: E402
from immustore_amd import _native as N  # noqa: E402

L = N.load()
ctx = m.Context(0)
for n in (1 << 20, 1 << 24):
    dig = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    N.check(L.mh_dev_fill_random(ctx.handle, dig.data_ptr(), dig.numel(), 5))
    lv = torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device="cuda")
    rt = torch.empty(32, dtype=torch.uint8, device="cuda")
    roots = {}
    for rep in range(3):
        for lpl in ("1", "2", "4"):
            os.environ["MH_DIGEST_LPL"] = lpl
            for _ in range(20):  # warm
                N.check(L.mh_dev_htree_build_digests(ctx.handle, dig.data_ptr(), n, lv.data_ptr(), rt.data_ptr()))
            ctx.synchronize()
            ctx.timing_reset()
            ctx.set_timing(True)
            k = 50 if n <= (1 << 20) else 10
            t0 = time.perf_counter()
            for _ in range(k):
                N.check(L.mh_dev_htree_build_digests(ctx.handle, dig.data_ptr(), n, lv.data_ptr(), rt.data_ptr()))
            ctx.synchronize()
            t = (time.perf_counter() - t0) / k
            ctx.set_timing(False)
            leaves = ctx.timing("leaves")[0] / k
            roots[lpl] = rt.cpu().numpy().tobytes()
            print(json.dumps({"n": n, "lpl": int(lpl), "rep": rep, "build_ms": round(t * 1e3, 4),
                              "leaves_ms": round(leaves, 4)}), flush=True)
    assert len(set(roots.values())) == 1
