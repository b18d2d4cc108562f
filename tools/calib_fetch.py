#!/usr/bin/env python3
"""FETCH_SIZE calibration for per-lane scattered window reads (the ragged
kernels' access pattern): k_sha_varlen over N messages of L bytes at stride L
(a known byte count, far past the 256 MiB Infinity Cache).  Profiled by
rocprofv3 --pmc FETCH_SIZE; compare the counter with N * L."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import immustore_amd as m
from immustore_amd import _native as N

n, L = 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda", 0)
ctx = m.Context(0, torch.cuda.current_stream(dev).cuda_stream)
lib = N.load()
buf = torch.empty(n * L + 16, dtype=torch.uint8, device=dev)
N.check(lib.mh_dev_fill_random(ctx.handle, buf.data_ptr(), buf.numel(), 9))
off = (torch.arange(n + 1, dtype=torch.int64, device=dev) * L).contiguous()
out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
for _ in range(3):
    N.check(lib.mh_dev_sha256_batch(ctx.handle, buf.data_ptr(), off.data_ptr(), n, out.data_ptr()))
torch.cuda.synchronize()
print("bytes", n * L)
