"""Python mirror of the reference's hot-path API over the C ABI.

Names and semantics follow the Go packages so that tests read like the
reference's own tests:

  embedded/htree   -> HTree (New / BuildWith / Root / InclusionProof),
                      InclusionProof, verify_inclusion(_batch)
  embedded/ahtree  -> AHtree (Append / RootAt / Root / InclusionProof /
                      ConsistencyProof / ResetSize / Size), and the
                      Verify*/Eval* functions of ahtree/verification.go
  embedded/store   -> build_hash_tree (value hash loop + Tx.BuildHashTree)

Every hash is computed by the HIP kernels of libimmustore_merkle.so.
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N

SHA256_SIZE = 32


def _addr(a):
    return None if a is None else a.ctypes.data


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def _digests(ds) -> np.ndarray:
    if isinstance(ds, np.ndarray):
        return np.ascontiguousarray(ds, dtype=np.uint8).reshape(-1, 32)
    if len(ds) == 0:
        return np.zeros((0, 32), np.uint8)
    return np.frombuffer(b"".join(bytes(d) for d in ds), dtype=np.uint8).reshape(-1, 32).copy()


def device_count() -> int:
    n = C.c_int(0)
    N.load().mh_device_count(C.byref(n))
    return n.value


class Context:
    """One HIP device + stream (mh_ctx)."""

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        self._lib = N.load()
        h = C.c_void_p()
        N.check(self._lib.mh_ctx_create(device, stream, C.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            self._lib.mh_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        N.check(self._lib.mh_ctx_synchronize(self.handle))

    @property
    def stream(self) -> int:
        return self._lib.mh_ctx_stream(self.handle)

    def set_timing(self, enable: bool):
        N.check(self._lib.mh_ctx_set_timing(self.handle, 1 if enable else 0))

    def timing(self, prefix: str = ""):
        ms = C.c_double(0)
        cnt = C.c_uint64(0)
        N.check(self._lib.mh_ctx_timing(self.handle, prefix.encode(), C.byref(ms), C.byref(cnt)))
        return ms.value, cnt.value

    def timing_reset(self):
        N.check(self._lib.mh_ctx_timing_reset(self.handle))


_default_ctx = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def levels_len(n: int) -> int:
    return N.load().mh_htree_levels_len(n)


def level_offset(n: int, level: int) -> int:
    return N.load().mh_htree_level_offset(n, level)


# --------------------------------------------------------------------- htree
@dataclass
class InclusionProof:
    """embedded/htree/htree.go:39-43."""
    leaf: int
    width: int
    terms: List[bytes] = field(default_factory=list)


class HTree:
    """embedded/htree/htree.go:32-37, backed by device-resident levels."""

    def __init__(self, max_width: int, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        self._lib = N.load()
        h = C.c_void_p()
        N.check(self._lib.mh_htree_new(self.ctx.handle, max_width, C.byref(h)))
        self.handle = h
        self.max_width = max_width

    @classmethod
    def New(cls, max_width: int, ctx: Optional[Context] = None) -> "HTree":
        return cls(max_width, ctx)

    def close(self):
        if self.handle:
            self._lib.mh_htree_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def build_with(self, digests) -> None:
        d = _digests(digests)
        N.check(self._lib.mh_htree_build_with(self.handle, _addr(d) if len(d) else None, d.shape[0]))

    BuildWith = build_with

    def build_entries(self, version: int, keys: Sequence[bytes], values: Sequence[bytes],
                      mds: Optional[Sequence[bytes]] = None, hval_overrides=None) -> np.ndarray:
        """Value hash loop + Tx.BuildHashTree; returns hVal per entry (n,32)."""
        n = len(keys)
        kb, ko = _csr(keys)
        vb, vo = _csr(values)
        mb = mo = None
        if mds is not None:
            mb, mo = _csr(mds)
        ov = use = None
        if hval_overrides is not None:
            ov = np.zeros((max(n, 1), 32), np.uint8)
            use = np.zeros(max(n, 1), np.uint8)
            for i, o in enumerate(hval_overrides):
                if o is not None:
                    ov[i] = np.frombuffer(bytes(o), np.uint8)
                    use[i] = 1
        hv = np.zeros((max(n, 1), 32), np.uint8)
        N.check(self._lib.mh_htree_build_entries(
            self.handle, version, n, _addr(kb), _addr(ko), _addr(mb), _addr(mo), _addr(vb),
            _addr(vo), _addr(ov), _addr(use), _addr(hv)))
        return hv[:n]

    def root(self) -> bytes:
        r = np.zeros(32, np.uint8)
        N.check(self._lib.mh_htree_root(self.handle, _addr(r)))
        return r.tobytes()

    Root = root

    @property
    def width(self) -> int:
        w = C.c_uint64(0)
        N.check(self._lib.mh_htree_width(self.handle, C.byref(w)))
        return w.value

    def inclusion_proof(self, i: int) -> InclusionProof:
        if i < 0:
            raise N.ErrIllegalArguments(N.MH_ERR_ILLEGAL_ARGUMENTS)
        terms = np.zeros((64, 32), np.uint8)
        nt = C.c_uint32(0)
        N.check(self._lib.mh_htree_inclusion_proof(self.handle, i, _addr(terms), 64, C.byref(nt)))
        return InclusionProof(i, self.width, [terms[k].tobytes() for k in range(nt.value)])

    InclusionProof = inclusion_proof

    def inclusion_proof_batch(self, leaves) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Device-generated InclusionProof for many leaves: (terms[n, max, 32],
        nterms[n], status[n]); terms in Go order."""
        lv = np.ascontiguousarray(leaves, np.uint64)
        n = lv.size
        mt = max(1, (max(self.width, 1) - 1).bit_length())
        terms = np.zeros((max(n, 1), mt, 32), np.uint8)
        nt = np.zeros(max(n, 1), np.uint32)
        st = np.zeros(max(n, 1), np.int32)
        N.check(self._lib.mh_htree_inclusion_proof_batch(self.handle, n, _addr(lv), _addr(terms),
                                                         mt, _addr(nt), _addr(st)))
        return terms[:n], nt[:n], st[:n]

    def inclusion_proof_pb_batch(self, leaves) -> Tuple[List[bytes], np.ndarray]:
        """InclusionProof protobuf messages (schema.proto:534, InclusionProofToProto
        database_protoconv.go:115-121) of many leaves, generated and encoded on
        the device -> (messages, status[n])."""
        lv = np.ascontiguousarray(leaves, np.uint64)
        return _pb_call(lambda out, cap, off, st: self._lib.mh_htree_inclusion_proof_pb_batch(
            self.handle, lv.size, _addr(lv), _addr(out), cap, _addr(off), _addr(st)), lv.size)

    def levels(self) -> np.ndarray:
        tot = levels_len(self.width)
        out = np.zeros((max(tot, 1), 32), np.uint8)
        N.check(self._lib.mh_htree_levels(self.handle, _addr(out), tot))
        return out[:tot]

    def levels_device_ptr(self) -> int:
        p = C.c_void_p()
        N.check(self._lib.mh_htree_levels_device(self.handle, C.byref(p)))
        return p.value


def _pb_call(call, n, guess: int = 0):
    """Run a packed-protobuf batch call, growing the output once on
    MH_ERR_BUFFER_TOO_SMALL -> (list of message bytes, status[n])."""
    off = np.zeros(n + 1, np.uint64)
    st = np.zeros(max(n, 1), np.int32)
    cap = guess or 2048 * max(n, 1)
    for _ in range(2):
        out = np.zeros(max(cap, 1), np.uint8)
        r = call(out, cap, off, st)
        if r == N.MH_ERR_BUFFER_TOO_SMALL:
            cap = int(off[n])
            continue
        N.check(r)
        return [out[off[k]:off[k + 1]].tobytes() for k in range(n)], st[:n]
    raise N.ErrBufferTooSmall(N.MH_ERR_BUFFER_TOO_SMALL)


def _csr(items):
    n = len(items)
    off = np.zeros(n + 1, np.uint64)
    if n:
        off[1:] = np.cumsum([len(x) for x in items])
    buf = np.frombuffer(b"".join(bytes(x) for x in items) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, off


def verify_inclusion_batch(proofs: Sequence[InclusionProof], digests, roots,
                           ctx: Optional[Context] = None) -> np.ndarray:
    """htree.VerifyInclusion (htree.go:166-195) for many proofs at once."""
    ctx = ctx or default_context()
    n = len(proofs)
    if n == 0:
        return np.zeros(0, bool)
    # Go ints: negative values travel as their 64-bit pattern
    leaf = np.array([p.leaf & 0xFFFFFFFFFFFFFFFF for p in proofs], np.uint64)
    width = np.array([p.width & 0xFFFFFFFFFFFFFFFF for p in proofs], np.uint64)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(p.terms) for p in proofs])
    terms = _digests([t for p in proofs for t in p.terms] or [b"\0" * 32])
    d = _digests(digests)
    r = _digests(roots)
    ok = np.zeros(n, np.uint8)
    N.check(N.load().mh_htree_verify_inclusion_batch(
        ctx.handle, n, _addr(leaf), _addr(width), _addr(off), _addr(terms), _addr(d), _addr(r),
        _addr(ok)))
    return ok.astype(bool)


def verify_inclusion(proof: Optional[InclusionProof], digest: bytes, root: bytes,
                     ctx: Optional[Context] = None) -> bool:
    """htree.VerifyInclusion: a nil proof does not verify (htree.go:167-169)."""
    if proof is None:
        return False
    return bool(verify_inclusion_batch([proof], [digest], [root], ctx)[0])


VerifyInclusion = verify_inclusion


def decode_inclusion_proof_pb(msgs, ctx: Optional[Context] = None):
    """InclusionProofFromProto (database_protoconv.go:123-129) over many
    encoded InclusionProof messages, on the device -> (status[n], proofs[n]);
    proofs[p] is an InclusionProof (Go int leaf / width, possibly negative)
    or None where status[p] is MH_ERR_CORRUPTED_DATA."""
    ctx = ctx or default_context()
    n = len(msgs)
    off = np.zeros(n + 1, np.uint64)
    if n:
        off[1:] = np.cumsum([len(x) for x in msgs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    leaf, width = np.zeros(max(n, 1), np.uint64), np.zeros(max(n, 1), np.uint64)
    to = np.zeros(n + 1, np.uint64)
    st = np.zeros(max(n, 1), np.int32)
    L = N.load()
    rc = L.mh_htree_inclusion_proof_pb_decode_batch(ctx.handle, n, _addr(buf), _addr(off),
                                                    _addr(leaf), _addr(width), _addr(to), None, 0,
                                                    _addr(st))
    if rc != N.MH_ERR_BUFFER_TOO_SMALL:
        N.check(rc)
    t = np.zeros((max(int(to[n]), 1), 32), np.uint8)
    N.check(L.mh_htree_inclusion_proof_pb_decode_batch(ctx.handle, n, _addr(buf), _addr(off),
                                                       _addr(leaf), _addr(width), _addr(to),
                                                       _addr(t), int(to[n]), _addr(st)))
    li, wi = leaf.view(np.int64), width.view(np.int64)
    proofs = [None if st[p] else InclusionProof(int(li[p]), int(wi[p]),
                                                [t[k].tobytes() for k in range(int(to[p]), int(to[p + 1]))])
              for p in range(n)]
    return st[:n], proofs


# -------------------------------------------------------------------- ahtree
class AHtree:
    """embedded/ahtree.AHtree with its dLog kept in HBM (in-memory; the pLog /
    cLog files stay with the Go appendables)."""

    def __init__(self, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        self._lib = N.load()
        h = C.c_void_p()
        N.check(self._lib.mh_ahtree_new(self.ctx.handle, C.byref(h)))
        self.handle = h

    def close(self):
        if self.handle:
            self._lib.mh_ahtree_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def append(self, d: Optional[bytes]):
        """ahtree.go:246-373 -> (n, h)."""
        if d is None:
            raise N.ErrIllegalArguments(N.MH_ERR_ILLEGAL_ARGUMENTS)
        p = _u8(d) if len(d) else np.zeros(1, np.uint8)
        n = C.c_uint64(0)
        h = np.zeros(32, np.uint8)
        N.check(self._lib.mh_ahtree_append(self.handle, _addr(p), len(d), C.byref(n), _addr(h)))
        return n.value, h.tobytes()

    Append = append

    def append_batch(self, payloads, with_roots: bool = False):
        p = np.ascontiguousarray(payloads, np.uint8)
        if p.ndim == 1:
            p = p.reshape(1, -1)
        m, plen = p.shape
        roots = np.zeros((max(m, 1), 32), np.uint8) if with_roots else None
        N.check(self._lib.mh_ahtree_append_batch(self.handle, _addr(p), m, plen, _addr(roots)))
        return roots[:m] if with_roots else None

    def append_batch_logs(self, payloads, p_off0: int = 0):
        """append_batch + the batch's pLog / cLog record streams (what
        (*AHtree).Append hands to t.pLog.Append / the cLog buffer,
        ahtree.go:266-282, 341-351) -> (plog bytes, clog bytes)."""
        p = np.ascontiguousarray(payloads, np.uint8)
        if p.ndim == 1:
            p = p.reshape(1, -1)
        m, plen = p.shape
        plog = np.zeros(max(1, m * (4 + plen)), np.uint8)
        clog = np.zeros(max(1, m * 12), np.uint8)
        N.check(self._lib.mh_ahtree_append_batch_logs(self.handle, _addr(p), m, plen, p_off0,
                                                      _addr(plog), _addr(clog), None))
        return plog[:m * (4 + plen)].tobytes(), clog[:m * 12].tobytes()

    def size(self) -> int:
        s = C.c_uint64(0)
        N.check(self._lib.mh_ahtree_size(self.handle, C.byref(s)))
        return s.value

    Size = size

    def root_at(self, n: int) -> bytes:
        r = np.zeros(32, np.uint8)
        N.check(self._lib.mh_ahtree_root_at(self.handle, n, _addr(r)))
        return r.tobytes()

    RootAt = root_at

    def root(self):
        n = C.c_uint64(0)
        r = np.zeros(32, np.uint8)
        N.check(self._lib.mh_ahtree_root(self.handle, C.byref(n), _addr(r)))
        return n.value, r.tobytes()

    Root = root

    def _proof(self, fn, i, j):
        t = np.zeros((256, 32), np.uint8)
        nt = C.c_uint32(0)
        N.check(fn(self.handle, i, j, _addr(t), 256, C.byref(nt)))
        return [t[k].tobytes() for k in range(nt.value)]

    def inclusion_proof(self, i: int, j: int) -> List[bytes]:
        return self._proof(self._lib.mh_ahtree_inclusion_proof, i, j)

    InclusionProof = inclusion_proof

    def consistency_proof(self, i: int, j: int) -> List[bytes]:
        return self._proof(self._lib.mh_ahtree_consistency_proof, i, j)

    ConsistencyProof = consistency_proof

    def proof_batch(self, kind: int, i, j, max_terms: int = 128):
        """Device-generated Inclusion (kind 0) / Consistency (kind 1) proofs for
        many (i, j): (terms[n, max_terms, 32], nterms[n], status[n])."""
        a = np.ascontiguousarray(i, np.uint64)
        b = np.ascontiguousarray(j, np.uint64)
        n = a.size
        terms = np.zeros((max(n, 1), max_terms, 32), np.uint8)
        nt = np.zeros(max(n, 1), np.uint32)
        st = np.zeros(max(n, 1), np.int32)
        N.check(self._lib.mh_ahtree_proof_batch(self.handle, kind, n, _addr(a), _addr(b),
                                                _addr(terms), max_terms, _addr(nt), _addr(st)))
        return terms[:n], nt[:n], st[:n]

    def dual_proof_v2_pb_batch(self, src_hdrs, tgt_hdrs, md_blob=b""):
        """ImmuStore.DualProofV2 (immustore.go:2356-2387) for many header pairs
        (TX_HEADER records, txlayer.py), each encoded on the device as the
        DualProofV2 protobuf message (schema.proto:437) -> (messages, status[n])."""
        from .txlayer import _blob, _hdrs
        s, t = _hdrs(src_hdrs), _hdrs(tgt_hdrs)
        bp, bl = _blob(md_blob)
        return _pb_call(lambda out, cap, off, st: self._lib.mh_ahtree_dual_proof_v2_pb_batch(
            self.handle, s.size, _addr(s), _addr(t), _addr(bp), bl, _addr(out), cap, _addr(off),
            _addr(st)), s.size)

    def reset_size(self, new_size: int):
        N.check(self._lib.mh_ahtree_reset_size(self.handle, new_size))

    ResetSize = reset_size

    def dlog(self, first: int = 0, count: Optional[int] = None) -> bytes:
        total = nodes_upto(self.size())
        if count is None:
            count = total - first
        out = np.zeros((max(count, 1), 32), np.uint8)
        N.check(self._lib.mh_ahtree_dlog(self.handle, first, count, _addr(out)))
        return out[:count].tobytes()


def nodes_upto(n: int) -> int:
    """ahtree.go:492-511."""
    return N.load().mh_ahtree_nodes_upto(n)


def _aht_batch(kind, items, ctx, want_eval=False):
    """items: (proof_terms, i, j, a, b)."""
    ctx = ctx or default_context()
    n = len(items)
    if n == 0:
        return np.zeros(0, bool), None
    vi = np.array([it[1] for it in items], np.uint64)
    vj = np.array([it[2] for it in items], np.uint64)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(it[0]) for it in items])
    terms = _digests([t for it in items for t in it[0]] or [b"\0" * 32])
    a = _digests([it[3] for it in items])
    b = _digests([it[4] for it in items])
    ok = np.zeros(n, np.uint8)
    ev = np.zeros((n, 64 if kind == N.MH_AHT_CONSISTENCY else 32), np.uint8) if want_eval else None
    N.check(N.load().mh_ahtree_verify_batch(ctx.handle, kind, n, _addr(vi), _addr(vj), _addr(off),
                                            _addr(terms), _addr(a), _addr(b), _addr(ok),
                                            _addr(ev)))
    return ok.astype(bool), ev


def ahtree_verify_inclusion(iproof, i, j, ileaf, jroot, ctx=None) -> bool:
    """ahtree/verification.go:21-30."""
    return bool(_aht_batch(N.MH_AHT_INCLUSION, [(iproof, i, j, ileaf, jroot)], ctx)[0][0])


def ahtree_eval_inclusion(iproof, i, j, ileaf, ctx=None) -> bytes:
    """ahtree/verification.go:32-56."""
    _, ev = _aht_batch(N.MH_AHT_INCLUSION, [(iproof, max(i, 1), max(j, i, 1), ileaf, b"\0" * 32)],
                       ctx, True)
    return ev[0].tobytes()


def ahtree_verify_consistency(cproof, i, j, iroot, jroot, ctx=None) -> bool:
    """ahtree/verification.go:58-70."""
    return bool(_aht_batch(N.MH_AHT_CONSISTENCY, [(cproof, i, j, iroot, jroot)], ctx)[0][0])


def ahtree_eval_consistency(cproof, i, j, ctx=None):
    """ahtree/verification.go:72-109 -> (ciRoot, cjRoot)."""
    if len(cproof) == 0:
        raise N.ErrIllegalArguments(N.MH_ERR_ILLEGAL_ARGUMENTS, "empty consistency proof")
    _, ev = _aht_batch(N.MH_AHT_CONSISTENCY, [(cproof, i, j, b"\0" * 32, b"\0" * 32)], ctx, True)
    return ev[0, :32].tobytes(), ev[0, 32:].tobytes()


def ahtree_verify_last_inclusion(iproof, i, leaf, root, ctx=None) -> bool:
    """ahtree/verification.go:111-118."""
    return bool(_aht_batch(N.MH_AHT_LAST_INCLUSION, [(iproof, i, i, leaf, root)], ctx)[0][0])


def ahtree_verify_batch(kind, items, ctx=None, want_eval=False):
    return _aht_batch(kind, items, ctx, want_eval)


# --------------------------------------------------------------------- store
def build_hash_tree(version: int, keys, values, mds=None, hval_overrides=None,
                    ctx: Optional[Context] = None):
    """immustore.go:1620-1632 + tx.go:332-355 for one transaction.

    Returns (Eh, hvals, levels)."""
    t = HTree(len(keys), ctx)
    try:
        hv = t.build_entries(version, keys, values, mds, hval_overrides)
        return t.root(), hv, t.levels()
    finally:
        t.close()


def verify_values(vals, off, hvals, vlen=None, ctx: Optional[Context] = None):
    """ImmuStore.readValueAt's integrity check (immustore.go:3235) over a
    batch (mh_verify_values_batch): value i = vals[off[i]:off[i+1]] (the bytes
    read), hvals (n, 32) the stored hVals, vlen (n,) the stored lengths (or
    None) -> (corrupted count, status int32[n]: 0 or MH_ERR_CORRUPTED_DATA)."""
    ctx = ctx or default_context()
    off = np.ascontiguousarray(off, np.uint64)
    n = len(off) - 1
    v = np.ascontiguousarray(vals, np.uint8)
    hv = np.ascontiguousarray(hvals, np.uint8)
    vl = None if vlen is None else np.ascontiguousarray(vlen, np.uint64)
    st = np.zeros(max(n, 1), np.int32)
    bad = C.c_uint64()
    N.check(N.load().mh_verify_values_batch(ctx.handle, n, _addr(v) if v.size else None,
                                            _addr(off), _addr(vl), _addr(hv), _addr(st),
                                            C.byref(bad)))
    return bad.value, st[:n]
