#!/usr/bin/env python3
"""Per-phase timing of k_txlog_wave over the last copy chunk's group of the a14
call (diagnosis): loads the `make WAVE_PROBE=1` build (build/probe/), runs the
bench's a14 log (2^16 records x 16 entries, pinned log and outputs) 30 times,
then once more with the stamps reset and prints, over the launch's waves, the
median / max time of each phase (100 MHz real-time counter) and the launch's
span from the first wave's start to the last wave's end.

    python3 tools/txlog_wave_probe.py
"""
import ctypes
import os
import struct
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MH_LIB_PATH", os.path.join(HERE, "build", "probe", "libimmustore_merkle.so"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import immustore_amd as m  # noqa: E402
from immustore_amd import _native as N  # noqa: E402
from immustore_amd.txlayer import TX_HEADER  # noqa: E402

PHASES = ("staging", "entry walk", "digests + leaves", "tree", "innerHash + Alh", "result staging",
          "stores")


def main():
    lib = N.load()
    probe = lib.mh_debug_txlog_wave_probe
    probe.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    ctx = m.Context(0)
    rng = np.random.default_rng(14)
    ntx, ne, kl = 1 << 16, 16, 16
    ent = 2 + 2 + kl + 4 + 8 + 32
    rec = 96 + ne * ent + 32
    buf = np.zeros((ntx, rec), np.uint8)
    buf[:, 0:8] = np.arange(1, ntx + 1, dtype=">u8").view(np.uint8).reshape(ntx, 8)
    buf[:, 24:88] = rng.integers(0, 256, (ntx, 64), dtype=np.uint8)
    buf[:, 89] = 1
    buf[:, 92:96] = np.frombuffer(struct.pack(">I", ne), np.uint8)
    e = buf[:, 96:96 + ne * ent].reshape(ntx, ne, ent)
    e[:, :, 3] = kl
    e[:, :, 4:4 + kl] = rng.integers(0, 256, (ntx, ne, kl), dtype=np.uint8)
    e[:, :, 4 + kl + 12:] = rng.integers(0, 256, (ntx, ne, 32), dtype=np.uint8)
    _, n, _, _, alh, _ = m.txlog_validate(buf.reshape(-1), ctx=ctx)
    buf[:, rec - 32:] = alh
    pin = torch.empty(buf.size, dtype=torch.uint8).pin_memory()
    pin.numpy()[:] = buf.reshape(-1)
    outs = (torch.empty(ntx * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER),
            torch.empty(ntx * 32, dtype=torch.uint8).pin_memory().numpy().reshape(ntx, 32),
            torch.empty(ntx, dtype=torch.int32).pin_memory().numpy())
    for _ in range(30):
        r = m.txlog_validate(pin.numpy(), ctx=ctx, out=outs)
        assert r[0] == 0 and r[1] == ntx and not r[5].any()
    assert probe(None, 0) == 0
    r = m.txlog_validate(pin.numpy(), ctx=ctx, out=outs)
    assert r[0] == 0 and r[1] == ntx and not r[5].any()
    nw = 8192
    st = np.zeros((nw, 8), np.uint64)
    assert probe(st.ctypes.data, nw) == 0
    st = st[st[:, 0] != 0].astype(np.int64)
    t0 = st[:, 0].min()
    us = (st - t0) / 100.0  # 100 MHz
    print("waves stamped: %d (the last group's launch)" % len(st))
    print("launch span: first start -> last end %.1f us; starts spread %.1f us; ends spread %.1f us"
          % (us[:, 7].max(), us[:, 0].max(), us[:, 7].max() - us[:, 7].min()))
    for k, name in enumerate(PHASES):
        d = us[:, k + 1] - us[:, k]
        print("%-18s median %6.1f us  p90 %6.1f  max %6.1f" % (name, np.median(d), np.percentile(d, 90), d.max()))
    tot = us[:, 7] - us[:, 0]
    print("%-18s median %6.1f us  max %6.1f" % ("wave total", np.median(tot), tot.max()))


if __name__ == "__main__":
    main()
