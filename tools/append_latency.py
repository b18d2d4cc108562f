#!/usr/bin/env python3
"""Latency of one (*AHtree).Append through mh_ahtree_append (H2D of the payload,
leaf / perfect / spine kernels, root back) vs the oracle on one host core."""
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
t = m.AHtree(ctx)
pay = orc.fill_random(32 * 200000, 9).reshape(-1, 32)
t.append_batch(pay[:100000])
o = orc.AHtree(200000)
o.append_batch(pay[:100000])
K = 2000
t0 = time.perf_counter()
for k in range(K):
    t.append(pay[100000 + k].tobytes())
t1 = time.perf_counter()
for k in range(K):
    o.append(pay[100000 + k].tobytes())
t2 = time.perf_counter()
assert t.root_at(100000 + K) == o.root_at(100000 + K)[1]
print('{"gpu_append_us": %.2f, "cpu_oracle_append_us": %.2f, "appends": %d}'
      % ((t1 - t0) / K * 1e6, (t2 - t1) / K * 1e6, K))
