#!/usr/bin/env python3
"""Times mh_txlog_validate on a 2^16-record x 16-entry log (pageable / pinned
input), its kernels (ctx timing) and a plain 75 MB host->device copy."""
import sys, time, numpy as np, struct, torch
sys.path.insert(0,'.')
import immustore_amd as m
ctx=m.Context(0)
rng=np.random.default_rng(14)
ntx,ne,kl=1<<16,16,16
ent=2+2+kl+4+8+32; hdr=8+8+8+32+32+2+2+4; rec=hdr+ne*ent+32
buf=np.zeros((ntx,rec),np.uint8)
buf[:,0:8]=np.arange(1,ntx+1,dtype='>u8').view(np.uint8).reshape(ntx,8)
buf[:,89]=1; buf[:,92:96]=np.frombuffer(struct.pack('>I',ne),np.uint8)
e=buf[:,hdr:hdr+ne*ent].reshape(ntx,ne,ent); e[:,:,3]=kl
raw=buf.reshape(-1).copy()
pin=torch.empty(raw.size,dtype=torch.uint8).pin_memory(); pr=pin.numpy(); pr[:]=raw
for name,x in (("pageable",raw),("pinned",pr),("pinned",pr)):  # warm-up calls
    t=time.perf_counter(); r=m.txlog_validate(x,ctx=ctx); t1=time.perf_counter()
    print(name, r[0], r[1], "%.3f ms"%((t1-t)*1e3), file=sys.stderr, flush=True)
from immustore_amd import _native as N
L = N.load()
for it in range(3):
    ctx.timing_reset(); ctx.set_timing(True)
    t=time.perf_counter(); r=m.txlog_validate(pr,ctx=ctx); t1=time.perf_counter()
    ctx.set_timing(False)
    ks = {k: round(ctx.timing(k)[0], 3) for k in ("txe_index","txe_assemble","sha256_csr","leaf_for","small_roots","tx_alh")}
    print("timed call %.3f ms" % ((t1-t)*1e3), ks, file=sys.stderr, flush=True)
d = torch.empty(pr.size, dtype=torch.uint8, device="cuda")
for it in range(3):
    torch.cuda.synchronize(); t=time.perf_counter()
    N.check(L.mh_memcpy_h2d(ctx.handle, d.data_ptr(), pr.ctypes.data, pr.size)); ctx.synchronize()
    print("h2d pinned 75MB %.3f ms" % ((time.perf_counter()-t)*1e3), file=sys.stderr, flush=True)
    t=time.perf_counter()
    N.check(L.mh_memcpy_h2d(ctx.handle, d.data_ptr(), raw.ctypes.data, raw.size)); ctx.synchronize()
    print("h2d pageable 75MB %.3f ms" % ((time.perf_counter()-t)*1e3), file=sys.stderr, flush=True)
