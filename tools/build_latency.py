#!/usr/bin/env python3
"""Latency of one (*HTree).BuildWith through mh_htree_build_with (digests from
host memory, levels kept on the device, root back) vs the oracle on one host
core, by width: where a size-based dispatch in the cgo shim should switch."""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "oracle"))
import torch  # noqa: F401,E402
import immustore_amd as m  # noqa: E402
import oracle as orc  # noqa: E402

ctx = m.Context(0)
out = {}
for w in (16, 256, 4096, 1 << 14, 1 << 16, 1 << 18, 1 << 20):
    d = orc.fill_random(32 * w, w).reshape(w, 32)
    t = m.HTree(w, ctx)
    t.build_with(d)
    K = max(3, min(500, (1 << 22) // w))
    t0 = time.perf_counter()
    for _ in range(K):
        t.build_with(d)
    t1 = time.perf_counter()
    for _ in range(max(1, K // 4)):
        _, r = orc.htree_build(d)
    t2 = time.perf_counter()
    assert r == t.root()
    out[w] = {"gpu_us": round((t1 - t0) / K * 1e6, 1),
              "cpu_us": round((t2 - t1) / max(1, K // 4) * 1e6, 1)}
print(json.dumps(out))
