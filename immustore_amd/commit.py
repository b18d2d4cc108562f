"""Python mirror of the commit path's hashing over many transactions
(C ABI mh_commit_pipe / mh_precommit_batch).

  ImmuStore.precommit / preCommitWith   immustore.go:1620-1632, 2301-2313
      hVal = SHA256(value) (EntrySpec.HashValue when IsValueTruncated), then
      Tx.BuildHashTree (tx.go:332-355) -> header Eh
  ReplicateTx Eh check                  immustore.go:1649-1654

A CommitPipe owns two HIP streams; a batch of transactions is hashed in
chunks whose host->device copies overlap the previous chunk's hashing.  A
CommitQueue (mh_commit_queue) coalesces single transactions submitted by many
threads -- the concurrent committers of precommit -- into such batches.  All
hashing runs in libimmustore_merkle.so; there is no CPU path.
"""
import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _native as N
from .merkle import Context, _addr, default_context


class EntrySpec:
    """embedded/store EntrySpec (immustore.go): key, KV metadata bytes,
    value, and HashValue for a truncated value."""

    __slots__ = ("key", "md", "value", "hash_value")

    def __init__(self, key: bytes, value: bytes = b"", md: bytes = b"",
                 hash_value: Optional[bytes] = None):
        self.key, self.value, self.md, self.hash_value = key, value, md, hash_value

    @property
    def is_value_truncated(self) -> bool:
        return self.hash_value is not None


def _csr(items):
    off = np.zeros(len(items) + 1, np.uint64)
    if items:
        off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    flat = b"".join(items)
    buf = np.frombuffer(flat, np.uint8).copy() if flat else None
    return buf, off


class CommitPipe:
    """mh_commit_pipe: per-goroutine (not synchronised)."""

    def __init__(self, ctx: Optional[Context] = None, chunk_bytes: int = 0):
        self.ctx = ctx or default_context()
        h = C.c_void_p()
        N.check(N.load().mh_commit_pipe_new(self.ctx.handle, chunk_bytes, C.byref(h)))
        self.handle = h.value

    def close(self):
        if self.handle:
            N.load().mh_commit_pipe_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def precommit_csr(self, version: int, tx_off, keys, key_off, vals, val_off, md=None,
                      md_off=None, hval_override=None, use_override=None, expect_eh=None,
                      max_width: int = 0, hvals_out=None, eh_out=None):
        """Raw CSR form (numpy arrays, possibly views of pinned memory).
        Returns (hvals [E,32], eh [ntx,32], status [ntx] int32)."""
        ntx = len(tx_off) - 1
        ne = int(tx_off[-1] - tx_off[0]) if ntx > 0 else 0
        hv = hvals_out if hvals_out is not None else np.zeros((max(ne, 1), 32), np.uint8)
        eh = eh_out if eh_out is not None else np.zeros((max(ntx, 1), 32), np.uint8)
        st = np.zeros(max(ntx, 1), np.int32)
        N.check(N.load().mh_precommit_batch(
            self.handle, version, max_width, ntx, _addr(tx_off), _addr(keys), _addr(key_off),
            _addr(md), _addr(md_off), _addr(vals), _addr(val_off), _addr(hval_override),
            _addr(use_override), _addr(expect_eh), _addr(hv), _addr(eh), _addr(st)))
        return hv[:ne], eh[:ntx], st[:ntx]

    def precommit(self, version: int, txs: Sequence[Sequence[EntrySpec]], expect_eh=None,
                  max_width: int = 0):
        """One Eh per transaction (list of EntrySpec).  Returns
        (hvals per tx as [n,32] arrays, eh [ntx,32], status [ntx])."""
        tx_off = np.zeros(len(txs) + 1, np.uint64)
        ents = []
        for t, es in enumerate(txs):
            ents.extend(es)
            tx_off[t + 1] = len(ents)
        keys, key_off = _csr([bytes(e.key) for e in ents])
        vals, val_off = _csr([bytes(e.value) for e in ents])
        mds = [bytes(e.md or b"") for e in ents]
        md, md_off = _csr(mds) if any(mds) else (None, None)
        ov = use = None
        if any(e.is_value_truncated for e in ents):
            ov = np.zeros((len(ents), 32), np.uint8)
            use = np.zeros(len(ents), np.uint8)
            for k, e in enumerate(ents):
                if e.is_value_truncated:
                    ov[k] = np.frombuffer(bytes(e.hash_value), np.uint8)
                    use[k] = 1
        exp = None
        if expect_eh is not None:
            exp = np.ascontiguousarray(np.asarray(expect_eh, np.uint8).reshape(-1, 32))
        hv, eh, st = self.precommit_csr(version, tx_off, keys, key_off, vals, val_off, md, md_off,
                                        ov, use, exp, max_width)
        per_tx = [hv[int(tx_off[t]):int(tx_off[t + 1])] for t in range(len(txs))]
        return per_tx, eh, st


class CommitQueue:
    """mh_commit_queue: group commit of single transactions from many threads
    (immustore.go:1620-1632 under MaxConcurrency committers).  submit() blocks
    until the transaction's hVals and Eh are ready; ctypes releases the GIL
    for the call, so Python threads wait concurrently."""

    def __init__(self, ctx: Optional[Context] = None, version: int = 1, max_width: int = 0,
                 max_txs: int = 64, wait_us: int = 50):
        self.ctx = ctx or default_context()
        h = C.c_void_p()
        N.check(N.load().mh_commit_queue_new(self.ctx.handle, version, max_width, max_txs,
                                             wait_us, C.byref(h)))
        self.handle = h.value

    def close(self):
        if self.handle:
            N.load().mh_commit_queue_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        b, t = C.c_uint64(), C.c_uint64()
        N.check(N.load().mh_commit_queue_stats(self.handle, C.byref(b), C.byref(t)))
        return b.value, t.value

    def submit_csr(self, keys, key_off, vals, val_off, md=None, md_off=None, hval_override=None,
                   use_override=None, expect_eh=None, hvals_out=None, eh_out=None):
        """One transaction in CSR form -> (status, hvals [n,32], eh bytes)."""
        n = len(key_off) - 1
        hv = hvals_out if hvals_out is not None else np.zeros((max(n, 1), 32), np.uint8)
        eh = eh_out if eh_out is not None else np.zeros(32, np.uint8)
        st = N.load().mh_commit_queue_submit(
            self.handle, n, _addr(keys), _addr(key_off), _addr(md), _addr(md_off), _addr(vals),
            _addr(val_off), _addr(hval_override), _addr(use_override), _addr(expect_eh),
            _addr(hv), _addr(eh))
        return st, hv[:n], bytes(eh)

    def submit(self, entries: Sequence[EntrySpec], expect_eh=None):
        """One transaction (list of EntrySpec) -> (status, hvals [n,32], eh)."""
        keys, key_off = _csr([bytes(e.key) for e in entries])
        vals, val_off = _csr([bytes(e.value) for e in entries])
        mds = [bytes(e.md or b"") for e in entries]
        md, md_off = _csr(mds) if any(mds) else (None, None)
        ov = use = None
        if any(e.is_value_truncated for e in entries):
            ov = np.zeros((len(entries), 32), np.uint8)
            use = np.zeros(len(entries), np.uint8)
            for k, e in enumerate(entries):
                if e.is_value_truncated:
                    ov[k] = np.frombuffer(bytes(e.hash_value), np.uint8)
                    use[k] = 1
        exp = np.frombuffer(bytes(expect_eh), np.uint8).copy() if expect_eh is not None else None
        return self.submit_csr(keys, key_off, vals, val_off, md, md_off, ov, use, exp)
