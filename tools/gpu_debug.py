#!/usr/bin/env python3
"""Stage-by-stage GPU vs oracle diagnostics (prints, never asserts)."""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402,F401
import immustore_amd as m  # noqa: E402
from immustore_amd import _native as N  # noqa: E402
import oracle as orc  # noqa: E402
from gpu_util import DevBuf  # noqa: E402


def H(b):
    return hashlib.sha256(b).digest()


def main():
    ctx = m.Context(0)
    L = N.load()
    # 1. generic SHA over a few ranges
    buf = orc.fill_random(5000, 7)
    cuts = np.array([0, 0, 1, 56, 120, 1144, 5000], np.uint64)
    db, do = DevBuf.from_host(ctx, buf), DevBuf.from_host(ctx, cuts)
    out = DevBuf(ctx, 32 * 6)
    N.check(L.mh_dev_sha256_batch(ctx.handle, db.ptr, do.ptr, 6, out.ptr))
    got = out.to_host().reshape(-1, 32)
    print("sha_csr:", [got[i].tobytes() == H(buf[int(cuts[i]):int(cuts[i + 1])].tobytes())
                       for i in range(6)])
    # 2. build_with (leaves from digests + reduce)
    for w in (1, 2, 3, 64, 1000):
        d = orc.fill_random(32 * w, 9).reshape(w, 32)
        t = m.HTree(w, ctx)
        t.build_with(d)
        lv, root = orc.htree_build(d)
        glv = t.levels()
        print("build_with w=%d root_ok=%s level0_ok=%s levels_ok=%s" % (
            w, t.root() == root, np.array_equal(glv[:w], lv[:w]), np.array_equal(glv, lv)))
    # 3. fixed entries, stage by stage
    for lpl in ("1", "2", "4"):
        os.environ["MH_LPL"] = lpl
        for n, vlen in ((64, 64), (64, 128), (64, 256), (1000, 256), (64, 1024), (64, 0), (64, 48)):
            vals = orc.fill_random(n * vlen, 1).reshape(n, vlen) if vlen else np.zeros((n, 0), np.uint8)
            keys = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).reshape(n, 8)
            dk = DevBuf.from_host(ctx, keys)
            dv = DevBuf.from_host(ctx, vals if vals.size else np.zeros(16, np.uint8))
            dl = DevBuf(ctx, m.levels_len(n) * 32)
            dh = DevBuf(ctx, n * 32)
            dr = DevBuf(ctx, 32)
            st = L.mh_dev_htree_build_entries_fixed(ctx.handle, 1, n, dk.ptr, 8, dv.ptr, vlen,
                                                    dh.ptr, dl.ptr, dr.ptr)
            ctx.synchronize()
            ohv, olv, oroot = orc.build_entries_fixed(1, keys, vals)
            hv = dh.to_host().reshape(-1, 32)
            lv = dl.to_host().reshape(-1, 32)
            hv_ok = [bool(np.array_equal(hv[i], ohv[i])) for i in range(n)]
            lv0_ok = [bool(np.array_equal(lv[i], olv[i])) for i in range(n)]
            print("fixed lpl=%s n=%d vlen=%d st=%d hv_ok=%d/%d leaf_ok=%d/%d levels_ok=%s root_ok=%s"
                  % (lpl, n, vlen, st, sum(hv_ok), n, sum(lv0_ok), n, np.array_equal(lv, olv),
                     dr.to_host().tobytes() == oroot))
            if sum(hv_ok) < n:
                bad = [i for i in range(n) if not hv_ok[i]][:8]
                print("   bad hv idx", bad)
                # is the device hash equal to the hash of some other value/offset?
                i = bad[0]
                cands = {H(vals[j].tobytes()): j for j in range(n)}
                print("   hv[%d] equals hash of value" % i, cands.get(hv[i].tobytes()))
    ctx.close()


if __name__ == "__main__":
    main()
