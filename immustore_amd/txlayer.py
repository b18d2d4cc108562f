"""Python mirror of the transaction layer around the Merkle path (embedded/store).

  TxHeader.Alh / innerHash         tx.go:249-319          -> tx_alh_batch
  Tx.BuildHashTree over many txs   tx.go:332-355          -> htree_build_many
  VerifyLinearProof                verification.go:40-64  -> verify_linear_proof_batch
  VerifyDualProofV2                verification.go:304-372 -> verify_dual_proof_v2_batch
  VerifyDualProof (v1, with linear / linear-advance parts)
                                   verification.go:127-235 -> verify_dual_proof_batch
  Tx.readFrom (read-path check)    tx.go:388-630          -> txlog_validate
  pkg/verification.VerifyDocument  verification.go:37-196 -> verify_document_batch

Headers travel as a numpy structured array of TX_HEADER (the C struct
mh_tx_header); metadata bytes live in a side blob addressed by md_off.
All hashing runs in libimmustore_merkle.so's HIP kernels.
"""
import ctypes as C
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .merkle import Context, _addr, _u8, default_context

TX_HEADER = np.dtype([("id", "<u8"), ("ts", "<i8"), ("bl_tx_id", "<u8"), ("bl_root", "u1", 32),
                      ("prev_alh", "u1", 32), ("eh", "u1", 32), ("version", "<u4"),
                      ("nentries", "<u4"), ("md_len", "<u4"), ("md_off", "<u4")])
assert TX_HEADER.itemsize == 136

# TxReader limits (store options: MaxTxEntries, MaxKeyLen; options.go)
DEFAULT_MAX_TX_ENTRIES = 1 << 10
DEFAULT_MAX_KEY_LEN = 1 << 10


def _ctx(ctx: Optional[Context]) -> Context:
    return ctx or default_context()


def _hdrs(h) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(h, TX_HEADER).reshape(-1))


def _blob(b) -> Tuple[Optional[np.ndarray], int]:
    if b is None or len(b) == 0:
        return None, 0
    a = _u8(b)
    return a, a.size


def _terms_csr(lists):
    off = np.zeros(len(lists) + 1, np.uint64)
    for k, t in enumerate(lists):
        off[k + 1] = off[k] + len(t)
    flat = b"".join(bytes(x) for t in lists for x in t)
    arr = np.frombuffer(flat, np.uint8).copy() if flat else np.zeros(32, np.uint8)
    return off, arr


def _d32(xs, n) -> np.ndarray:
    if isinstance(xs, np.ndarray):
        a = np.ascontiguousarray(xs, np.uint8).reshape(-1, 32)
    else:
        a = np.frombuffer(b"".join(bytes(x) for x in xs), np.uint8).reshape(-1, 32).copy() \
            if n else np.zeros((0, 32), np.uint8)
    assert a.shape[0] == n
    return a


def tx_alh_batch(hdrs, md_blob=b"", ctx: Optional[Context] = None):
    """-> (inner[n,32], alh[n,32]) for every header (TxHeader.Alh, tx.go:307)."""
    h = _hdrs(hdrs)
    n = h.size
    inner = np.zeros((max(n, 1), 32), np.uint8)
    alh = np.zeros((max(n, 1), 32), np.uint8)
    mb, ml = _blob(md_blob)
    N.check(N.load().mh_tx_alh_batch(_ctx(ctx).handle, n, _addr(h), _addr(mb), ml, _addr(inner),
                                     _addr(alh)))
    return inner[:n], alh[:n]


def htree_build_many(trees: Sequence, ctx: Optional[Context] = None) -> np.ndarray:
    """One htree root per digest list (width 0 -> SHA256(nil))."""
    off = np.zeros(len(trees) + 1, np.uint64)
    for k, t in enumerate(trees):
        off[k + 1] = off[k] + len(t)
    flat = b"".join(bytes(d) for t in trees for d in t)
    d = np.frombuffer(flat, np.uint8).copy() if flat else None
    roots = np.zeros((max(len(trees), 1), 32), np.uint8)
    N.check(N.load().mh_htree_build_many(_ctx(ctx).handle, len(trees), _addr(off), _addr(d),
                                         _addr(roots)))
    return roots[:len(trees)]


def verify_linear_proof_batch(proofs, ctx: Optional[Context] = None) -> np.ndarray:
    """proofs: sequence of (proof_src, proof_tgt, terms, src, tgt, src_alh, tgt_alh)."""
    n = len(proofs)
    if n == 0:
        return np.zeros(0, bool)
    ps = np.array([p[0] for p in proofs], np.uint64)
    pt = np.array([p[1] for p in proofs], np.uint64)
    off, terms = _terms_csr([p[2] for p in proofs])
    s = np.array([p[3] for p in proofs], np.uint64)
    t = np.array([p[4] for p in proofs], np.uint64)
    sa = _d32([p[5] for p in proofs], n)
    ta = _d32([p[6] for p in proofs], n)
    ok = np.zeros(n, np.uint8)
    N.check(N.load().mh_verify_linear_proof_batch(_ctx(ctx).handle, n, _addr(ps), _addr(pt),
                                                  _addr(off), _addr(terms), _addr(s), _addr(t),
                                                  _addr(sa), _addr(ta), _addr(ok)))
    return ok.astype(bool)


def verify_dual_proof_v2_batch(src_hdrs, tgt_hdrs, md_blob, incl, cons, src, tgt, src_alh,
                               tgt_alh, ctx: Optional[Context] = None) -> np.ndarray:
    """status[n] (0 = verifies, else the MH_ERR_* of the Go error)."""
    sh, th = _hdrs(src_hdrs), _hdrs(tgt_hdrs)
    n = sh.size
    if n == 0:
        return np.zeros(0, np.int32)
    mb, ml = _blob(md_blob)
    io, it = _terms_csr(incl)
    co, ct = _terms_csr(cons)
    s = np.asarray(src, np.uint64)
    t = np.asarray(tgt, np.uint64)
    sa, ta = _d32(src_alh, n), _d32(tgt_alh, n)
    st = np.zeros(n, np.int32)
    N.check(N.load().mh_verify_dual_proof_v2_batch(
        _ctx(ctx).handle, n, _addr(sh), _addr(th), _addr(mb), ml, _addr(io), _addr(it),
        _addr(co), _addr(ct), _addr(s), _addr(t), _addr(sa), _addr(ta), _addr(st)))
    return st


def VerifyDualProofV2(src_hdr, tgt_hdr, md_blob, incl, cons, src, tgt, src_alh, tgt_alh,
                      ctx: Optional[Context] = None) -> None:
    """Go-shaped single proof: raises the Go error, returns None on success."""
    st = verify_dual_proof_v2_batch([src_hdr], [tgt_hdr], md_blob, [incl], [cons], [src], [tgt],
                                    [src_alh], [tgt_alh], ctx)
    N.check(int(st[0]))


class _DualProofBatch(C.Structure):
    """mirror of mh_dual_proof_batch (include/immustore_merkle.h)"""
    _fields_ = [("n", C.c_uint64), ("src_hdr", C.c_void_p), ("tgt_hdr", C.c_void_p),
                ("md_blob", C.c_void_p), ("md_blob_len", C.c_uint64),
                ("incl_off", C.c_void_p), ("incl_terms", C.c_void_p),
                ("cons_off", C.c_void_p), ("cons_terms", C.c_void_p),
                ("target_bl_tx_alh", C.c_void_p), ("last_off", C.c_void_p),
                ("last_terms", C.c_void_p), ("has_linear", C.c_void_p),
                ("linear_src", C.c_void_p), ("linear_tgt", C.c_void_p),
                ("linear_off", C.c_void_p), ("linear_terms", C.c_void_p),
                ("has_advance", C.c_void_p), ("advance_off", C.c_void_p),
                ("advance_terms", C.c_void_p), ("advance_incl_first", C.c_void_p),
                ("advance_incl_off", C.c_void_p), ("advance_incl_terms", C.c_void_p),
                ("src", C.c_void_p), ("tgt", C.c_void_p), ("src_alh", C.c_void_p),
                ("tgt_alh", C.c_void_p)]


def verify_dual_proof_batch(src_hdrs, tgt_hdrs, md_blob, incl, cons, target_bl_tx_alh, last,
                            linear, advance, src, tgt, src_alh, tgt_alh,
                            ctx: Optional[Context] = None) -> np.ndarray:
    """VerifyDualProof (v1, verification.go:127-235) over n proofs -> ok[n] (bool).

    linear[p]: None (nil proof) or (SourceTxID, TargetTxID, terms);
    advance[p]: None or (LinearProofTerms, [InclusionProofs...])."""
    sh, th = _hdrs(src_hdrs), _hdrs(tgt_hdrs)
    n = sh.size
    if n == 0:
        return np.zeros(0, bool)
    keep = []

    def k(a):
        keep.append(a)
        return _addr(a)

    mb, ml = _blob(md_blob)
    io, it = _terms_csr(incl)
    co, ct = _terms_csr(cons)
    lo, lt = _terms_csr(last)
    has_lin = np.array([x is not None for x in linear], np.uint8)
    lsrc = np.array([x[0] if x is not None else 0 for x in linear], np.uint64)
    ltgt = np.array([x[1] if x is not None else 0 for x in linear], np.uint64)
    lno, lnt = _terms_csr([x[2] if x is not None else [] for x in linear])
    has_adv = np.array([x is not None for x in advance], np.uint8)
    ao, at = _terms_csr([x[0] if x is not None else [] for x in advance])
    nested = [x[1] if x is not None else [] for x in advance]
    first = np.zeros(n + 1, np.uint64)
    for p, ns in enumerate(nested):
        first[p + 1] = first[p] + len(ns)
    qo, qt = _terms_csr([ip for ns in nested for ip in ns])
    s_ = np.asarray(src, np.uint64)
    t_ = np.asarray(tgt, np.uint64)
    sa, ta, tba = _d32(src_alh, n), _d32(tgt_alh, n), _d32(target_bl_tx_alh, n)
    b = _DualProofBatch(n, k(sh), k(th), k(mb) if mb is not None else None, ml, k(io), k(it),
                        k(co), k(ct), k(tba), k(lo), k(lt), k(has_lin), k(lsrc), k(ltgt), k(lno),
                        k(lnt), k(has_adv), k(ao), k(at), k(first), k(qo), k(qt), k(s_), k(t_),
                        k(sa), k(ta))
    ok = np.zeros(n, np.uint8)
    N.check(N.load().mh_verify_dual_proof_batch(_ctx(ctx).handle, C.byref(b), _addr(ok)))
    return ok.astype(bool)


class _DocumentBatch(C.Structure):
    """mirror of mh_document_batch (include/immustore_merkle.h)"""
    _fields_ = [("n", C.c_uint64), ("doc", C.c_void_p), ("doc_off", C.c_void_p),
                ("doc_key", C.c_void_p), ("doc_key_off", C.c_void_p), ("tx_hdr", C.c_void_p),
                ("ent_off", C.c_void_p), ("ekeys", C.c_void_p), ("ekey_off", C.c_void_p),
                ("emd", C.c_void_p), ("emd_off", C.c_void_p), ("ehval", C.c_void_p),
                ("src_hdr", C.c_void_p), ("tgt_hdr", C.c_void_p), ("md_blob", C.c_void_p),
                ("md_blob_len", C.c_uint64), ("incl_off", C.c_void_p),
                ("incl_terms", C.c_void_p), ("cons_off", C.c_void_p),
                ("cons_terms", C.c_void_p), ("known_tx_id", C.c_void_p),
                ("known_alh", C.c_void_p)]


def _csr_bytes(items):
    off = np.zeros(len(items) + 1, np.uint64)
    for k, b in enumerate(items):
        off[k + 1] = off[k] + len(b)
    flat = b"".join(bytes(b) for b in items)
    return off, (np.frombuffer(flat, np.uint8).copy() if flat else np.zeros(16, np.uint8))


def verify_document_batch(docs, ctx: Optional[Context] = None):
    """pkg/verification.VerifyDocument (verification.go:37-196), hashing part,
    for many documents.  docs: sequence of dicts with
      encoded_document (bytes), doc_key (bytes, encodedKeyForDocument),
      tx_hdr (TX_HEADER record), entries [(key, md_bytes, hvalue), ...],
      src_hdr, tgt_hdr (TX_HEADER records), incl, cons (term lists),
      known_tx_id (int, 0 = none), known_alh (32 bytes);
    plus md_blob under key "md_blob" of the FIRST dict (shared by all headers).
    -> (status[n] int32, target_alh[n,32])."""
    n = len(docs)
    if n == 0:
        return np.zeros(0, np.int32), np.zeros((0, 32), np.uint8)
    b, keep = pack_document_batch(docs)
    return call_document_batch(b, n, ctx)


def call_document_batch(b, n, ctx: Optional[Context] = None):
    """mh_verify_document_batch over a batch packed by pack_document_batch."""
    st = np.zeros(n, np.int32)
    alh = np.zeros((n, 32), np.uint8)
    N.check(N.load().mh_verify_document_batch(_ctx(ctx).handle, C.byref(b), _addr(st),
                                              _addr(alh)))
    return st, alh


class _Pinned:
    """A numpy array in pinned host memory (mh_host_alloc_pinned)."""

    def __init__(self, a):
        a = np.ascontiguousarray(a)
        self.p = C.c_void_p()
        N.check(N.load().mh_host_alloc_pinned(max(a.nbytes, 1), C.byref(self.p)))
        buf = (C.c_uint8 * max(a.nbytes, 1)).from_address(self.p.value)
        self.a = np.frombuffer(buf, np.uint8, count=a.nbytes).view(a.dtype).reshape(a.shape)
        self.a[...] = a

    def __del__(self):
        if self.p:
            N.load().mh_host_free_pinned(self.p)
            self.p = None


class _Arena:
    """Arrays packed back to back (256-byte aligned) in ONE pinned host
    allocation, as a cgo shim's packing arena holds a batch."""

    def __init__(self, arrays):
        arrays = [np.ascontiguousarray(a) for a in arrays]
        offs, o = [], 0
        for a in arrays:
            offs.append(o)
            o += (max(a.nbytes, 1) + 255) & ~255
        self.p = C.c_void_p()
        N.check(N.load().mh_host_alloc_pinned(max(o, 1), C.byref(self.p)))
        self.addrs = []
        for a, off in zip(arrays, offs):
            if a.nbytes:
                C.memmove(self.p.value + off, a.ctypes.data, a.nbytes)
            self.addrs.append(self.p.value + off)

    def __del__(self):
        if self.p:
            N.load().mh_host_free_pinned(self.p)
            self.p = None


def pack_document_batch(docs, pinned=False):
    """The mh_document_batch of verify_document_batch's docs -> (struct, the
    arrays it points into, to be kept alive while it is used).  pinned: True
    puts every array in its own pinned allocation; "arena" packs them all into
    one pinned allocation, as a cgo shim's packing arena would."""
    n = len(docs)
    keep = []
    arena = []

    def k(a):
        if pinned == "arena":
            arena.append(np.ascontiguousarray(a))
            return len(arena) - 1  # an index until the arena exists
        if pinned:
            a = _Pinned(a)
            keep.append(a)
            return a.a.ctypes.data
        keep.append(a)
        return _addr(a)

    doff, dbuf = _csr_bytes([d["encoded_document"] for d in docs])
    koff, kbuf = _csr_bytes([d["doc_key"] for d in docs])
    txh = _hdrs([d["tx_hdr"] for d in docs])
    ents = [e for d in docs for e in d["entries"]]
    ent_off = np.zeros(n + 1, np.uint64)
    for i, d in enumerate(docs):
        ent_off[i + 1] = ent_off[i] + len(d["entries"])
    ekoff, ekbuf = _csr_bytes([e[0] for e in ents])
    emoff, embuf = _csr_bytes([e[1] for e in ents])
    ehv = _d32([e[2] for e in ents], len(ents)) if ents else np.zeros((1, 32), np.uint8)
    sh = _hdrs([d["src_hdr"] for d in docs])
    th = _hdrs([d["tgt_hdr"] for d in docs])
    mb, ml = _blob(docs[0].get("md_blob", b""))
    io, it = _terms_csr([d["incl"] for d in docs])
    co, ct = _terms_csr([d["cons"] for d in docs])
    kid = np.array([d.get("known_tx_id", 0) for d in docs], np.uint64)
    kalh = _d32([d.get("known_alh", bytes(32)) for d in docs], n)
    ptrs = [k(dbuf), k(doff), k(kbuf), k(koff), k(txh), k(ent_off), k(ekbuf), k(ekoff), k(embuf),
            k(emoff), k(ehv), k(sh), k(th), k(mb) if mb is not None else None, ml, k(io), k(it),
            k(co), k(ct), k(kid), k(kalh)]
    if pinned == "arena":
        ar = _Arena(arena)
        keep.append(ar)
        ptrs = [p if i == 14 or p is None else ar.addrs[p] for i, p in enumerate(ptrs)]
    b = _DocumentBatch(n, *ptrs)
    return b, keep


def txlog_validate(buf, max_entries: int = DEFAULT_MAX_TX_ENTRIES,
                   max_key_len: int = DEFAULT_MAX_KEY_LEN, max_txs: Optional[int] = None,
                   ctx: Optional[Context] = None, out=None, dev: Optional[int] = None):
    """-> (status, ntx, consumed, hdrs[ntx] TX_HEADER (Eh rebuilt), alh[ntx,32], per_tx[ntx])

    dev: the device address of the same bytes already resident on the
    context's device (mh_txlog_validate_resident: no host->device copy; the
    allocation must extend 256 bytes past the log)

    status is the structural error that stopped parsing (0 at a clean end);
    per_tx[k] is 0 or MH_ERR_CORRUPTED_DATA (ALH mismatch).

    out: optional (hdrs, alh, per_tx) arrays kept by the caller across calls
    (e.g. in pinned memory, as a cgo shim keeps its arena); hdrs may be None
    when the headers are not wanted.  Their length caps the records read."""
    b = _u8(buf)
    cap = max(1, len(b) // 122 + 1)  # a record is >= 122 bytes (90 + 32)
    if max_txs is not None:
        cap = max(1, min(cap, max_txs))
    if out is not None:
        hd, alh, sts = out
        cap = max(1, min(cap, len(alh), len(sts), len(hd) if hd is not None else cap))
        assert alh.dtype == np.uint8 and alh.shape[1:] == (32,) and sts.dtype == np.int32
        assert hd is None or hd.dtype == TX_HEADER
        assert all(a is None or a.flags.c_contiguous for a in out)
    else:
        # outputs are written for the parsed records only: no zero fill, and
        # the results are returned as views (no copies of the unused capacity)
        hd = np.empty(cap, TX_HEADER)
        alh = np.empty((cap, 32), np.uint8)
        sts = np.empty(cap, np.int32)
    ntx, used = C.c_uint64(0), C.c_uint64(0)
    lim = cap if max_txs is None else min(cap, max_txs)
    if dev is None:
        rc = N.load().mh_txlog_validate(_ctx(ctx).handle, _addr(b) if b.size else None, b.size,
                                        max_entries, max_key_len, lim, C.byref(ntx),
                                        C.byref(used), _addr(hd) if hd is not None else None,
                                        _addr(alh), _addr(sts))
    else:
        rc = N.load().mh_txlog_validate_resident(
            _ctx(ctx).handle, _addr(b) if b.size else None, dev, b.size, max_entries, max_key_len,
            lim, C.byref(ntx), C.byref(used), _addr(hd) if hd is not None else None, _addr(alh),
            _addr(sts))
    if rc < 0:
        N.check(rc)
    k = ntx.value
    return rc, k, used.value, (hd[:k] if hd is not None else None), alh[:k], sts[:k]


def txlog_validate_clog(dev, length: Optional[int], clog, ntx: Optional[int] = None,
                        clog_entry_size: int = 12, max_entries: int = DEFAULT_MAX_TX_ENTRIES,
                        max_key_len: int = DEFAULT_MAX_KEY_LEN, ctx: Optional[Context] = None,
                        out=None, clog_dev: Optional[int] = None):
    """mh_txlog_validate_clog: readTx (immustore.go:3048-3060) of txs 1..ntx of
    a tx log already on the device (dev: its address, length bytes, the
    allocation 256 bytes longer) or in host memory (dev: a bytes-like / numpy
    buffer, pinned or not; length None or at most its size), located by the
    commit-log entries clog
    (bytes, 12 or 44 per tx; or clog_dev: their device address with ntx)
    -> (status, nbad, first_bad, hdrs[ntx] TX_HEADER, alh[ntx,32], per_tx[ntx]).

    out: optional (hdrs, alh, per_tx) arrays (host numpy, pinned or not), or
    (hdrs_addr, alh_addr, per_tx_addr) device addresses (ints; any may be None)
    -- then the arrays returned are None."""
    if not isinstance(dev, int):
        hb = _u8(dev)
        length = hb.size if length is None else length
        assert length <= hb.size
        dev = _addr(hb) if hb.size else None
    if clog_dev is None:
        cb = _u8(clog)
        n = len(cb) // clog_entry_size if ntx is None else ntx
        assert len(cb) >= n * clog_entry_size
        caddr = _addr(cb) if cb.size else None
    else:
        assert ntx is not None
        n, caddr = ntx, clog_dev
    nbad, first = C.c_uint64(0), C.c_uint64(0)
    if out is not None and all(x is None or isinstance(x, int) for x in out):
        ptrs, arrs = list(out), (None, None, None)
    else:
        if out is not None:
            hd, alh, sts = out
            assert len(alh) >= n and len(sts) >= n and (hd is None or len(hd) >= n)
        else:
            hd = np.empty(max(n, 1), TX_HEADER)
            alh = np.empty((max(n, 1), 32), np.uint8)
            sts = np.empty(max(n, 1), np.int32)
        ptrs = [_addr(hd) if hd is not None else None, _addr(alh), _addr(sts)]
        arrs = (hd[:n] if hd is not None else None, alh[:n], sts[:n])
    rc = N.load().mh_txlog_validate_clog(_ctx(ctx).handle, dev, length, caddr, n, clog_entry_size,
                                         max_entries, max_key_len, ptrs[0], ptrs[1], ptrs[2],
                                         C.byref(nbad), C.byref(first))
    if rc < 0:
        N.check(rc)
    return (rc, nbad.value, first.value) + arrs


def txlog_scan(buf, max_entries: int = DEFAULT_MAX_TX_ENTRIES,
               max_key_len: int = DEFAULT_MAX_KEY_LEN, max_txs: Optional[int] = None):
    """Record structure only (host, no device) -> (status, ntx, consumed,
    hdrs[ntx] TX_HEADER with eh zero, alh_off[ntx])."""
    b = _u8(buf)
    cap = max(1, len(b) // 122 + 1)
    if max_txs is not None:
        cap = max(1, min(cap, max_txs))
    hd = np.zeros(cap, TX_HEADER)
    ao = np.zeros(cap, np.uint64)
    ntx, used = C.c_uint64(0), C.c_uint64(0)
    rc = N.load().mh_txlog_scan(_addr(b) if b.size else None, b.size, max_entries, max_key_len,
                                cap if max_txs is None else min(cap, max_txs), C.byref(ntx),
                                C.byref(used), _addr(hd), _addr(ao))
    if rc < 0:
        N.check(rc)
    k = ntx.value
    return rc, k, used.value, hd[:k], ao[:k]


def decode_dual_proof_v2_pb(msgs, ctx: Optional[Context] = None):
    """DualProofV2FromProto (database_protoconv.go:226-262) over many encoded
    DualProofV2 messages, on the device -> (status[n], src TX_HEADER[n],
    tgt TX_HEADER[n], md_blob, incl_off, incl_terms, cons_off, cons_terms);
    the outputs are mh_verify_dual_proof_v2_batch's arguments."""
    n = len(msgs)
    off = np.zeros(n + 1, np.uint64)
    if n:
        off[1:] = np.cumsum([len(x) for x in msgs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    sh = np.zeros(max(n, 1), TX_HEADER)
    th = np.zeros(max(n, 1), TX_HEADER)
    md = np.zeros(max(2 * n * 268, 1), np.uint8)
    io = np.zeros(n + 1, np.uint64)
    co = np.zeros(n + 1, np.uint64)
    st = np.zeros(max(n, 1), np.int32)
    L = N.load()
    h = _ctx(ctx).handle
    rc = L.mh_dual_proof_v2_pb_decode_batch(h, n, _addr(buf), _addr(off), _addr(sh), _addr(th),
                                            _addr(md), _addr(io), None, 0, _addr(co), None, 0,
                                            _addr(st))
    if rc not in (0, 19):  # MH_ERR_BUFFER_TOO_SMALL: the size query
        N.check(rc)
    it = np.zeros((max(int(io[n]), 1), 32), np.uint8)
    ct = np.zeros((max(int(co[n]), 1), 32), np.uint8)
    N.check(L.mh_dual_proof_v2_pb_decode_batch(h, n, _addr(buf), _addr(off), _addr(sh), _addr(th),
                                               _addr(md), _addr(io), _addr(it), int(io[n]),
                                               _addr(co), _addr(ct), int(co[n]), _addr(st)))
    return st[:n], sh[:n], th[:n], md.tobytes(), io, it[:int(io[n])], co, ct[:int(co[n])]


class _DualProofDecoded(C.Structure):
    """mirror of mh_dual_proof_decoded (include/immustore_merkle.h)"""
    _fields_ = [(f, C.c_void_p) for f in (
        "src_hdr", "tgt_hdr", "md_blob", "target_bl_tx_alh", "has_linear", "linear_src",
        "linear_tgt", "has_advance", "incl_off", "cons_off", "last_off", "linear_off",
        "advance_off", "advance_incl_first", "advance_incl_off", "incl_terms", "cons_terms",
        "last_terms", "linear_terms", "advance_terms", "advance_incl_terms")] + \
        [(f, C.c_uint64) for f in ("incl_cap", "cons_cap", "last_cap", "linear_cap", "advance_cap",
                                   "advance_incl_cap", "advance_incl_terms_cap", "nested_proofs",
                                   "nested_terms")]


_TERM_LISTS = ("incl", "cons", "last", "linear", "advance")


def decode_dual_proof_pb(msgs, ctx: Optional[Context] = None):
    """DualProofFromProto (v1, database_protoconv.go:213-287) over many encoded
    DualProof messages, on the device -> (status[n], dict of the
    mh_dual_proof_batch arrays: src_hdr, tgt_hdr, md_blob, target_bl_tx_alh,
    has_linear, linear_src, linear_tgt, has_advance, <list>_off / <list>_terms
    for incl, cons, last, linear, advance, advance_incl_first,
    advance_incl_off, advance_incl_terms)."""
    n = len(msgs)
    off = np.zeros(n + 1, np.uint64)
    if n:
        off[1:] = np.cumsum([len(x) for x in msgs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    m = max(n, 1)
    a = {"src_hdr": np.zeros(m, TX_HEADER), "tgt_hdr": np.zeros(m, TX_HEADER),
         "md_blob": np.zeros(max(2 * n * 268, 1), np.uint8),
         "target_bl_tx_alh": np.zeros((m, 32), np.uint8), "has_linear": np.zeros(m, np.uint8),
         "linear_src": np.zeros(m, np.uint64), "linear_tgt": np.zeros(m, np.uint64),
         "has_advance": np.zeros(m, np.uint8), "advance_incl_first": np.zeros(n + 1, np.uint64),
         "advance_incl_off": np.zeros(1, np.uint64)}
    for t in _TERM_LISTS:
        a[t + "_off"] = np.zeros(n + 1, np.uint64)
    st = np.zeros(m, np.int32)
    L, h = N.load(), _ctx(ctx).handle

    def call(caps):
        for t in _TERM_LISTS + ("advance_incl",):
            a[t + "_terms"] = np.zeros((max(caps.get(t, 0), 1), 32), np.uint8)
        a["advance_incl_off"] = np.zeros(caps.get("nested", 0) + 1, np.uint64)
        d = _DualProofDecoded(*[_addr(a[f]) for f, _ in _DualProofDecoded._fields_[:21]],
                              *[caps.get(t, 0) for t in _TERM_LISTS],
                              caps.get("nested", 0), caps.get("advance_incl", 0), 0, 0)
        rc = L.mh_dual_proof_pb_decode_batch(h, n, _addr(buf), _addr(off), C.byref(d), _addr(st))
        return rc, d

    rc, d = call({})
    if rc == N.MH_ERR_BUFFER_TOO_SMALL:
        caps = {t: int(a[t + "_off"][n]) for t in _TERM_LISTS}
        caps["nested"], caps["advance_incl"] = int(d.nested_proofs), int(d.nested_terms)
        rc, d = call(caps)
    N.check(rc)
    for t in _TERM_LISTS:
        a[t + "_terms"] = a[t + "_terms"][:int(a[t + "_off"][n])]
    a["advance_incl_terms"] = a["advance_incl_terms"][:int(d.nested_terms)]
    for f in ("src_hdr", "tgt_hdr", "target_bl_tx_alh", "has_linear", "linear_src", "linear_tgt",
              "has_advance"):
        a[f] = a[f][:n]
    return st[:n], a


def verify_decoded_dual_proof_batch(dec, src, tgt, src_alh, tgt_alh,
                                    ctx: Optional[Context] = None) -> np.ndarray:
    """VerifyDualProof (v1) straight over decode_dual_proof_pb's arrays -> ok[n]."""
    n = dec["src_hdr"].size
    if n == 0:
        return np.zeros(0, bool)
    keep = []

    def k(x):
        x = np.ascontiguousarray(x) if len(x) else np.zeros(32, np.uint8)
        keep.append(x)
        return _addr(x)

    s_, t_ = np.asarray(src, np.uint64), np.asarray(tgt, np.uint64)
    sa, ta = _d32(src_alh, n), _d32(tgt_alh, n)
    b = _DualProofBatch(n, k(dec["src_hdr"]), k(dec["tgt_hdr"]), k(dec["md_blob"]),
                        dec["md_blob"].size, k(dec["incl_off"]), k(dec["incl_terms"]),
                        k(dec["cons_off"]), k(dec["cons_terms"]), k(dec["target_bl_tx_alh"]),
                        k(dec["last_off"]), k(dec["last_terms"]), k(dec["has_linear"]),
                        k(dec["linear_src"]), k(dec["linear_tgt"]), k(dec["linear_off"]),
                        k(dec["linear_terms"]), k(dec["has_advance"]), k(dec["advance_off"]),
                        k(dec["advance_terms"]), k(dec["advance_incl_first"]),
                        k(dec["advance_incl_off"]), k(dec["advance_incl_terms"]), k(s_), k(t_),
                        k(sa), k(ta))
    ok = np.zeros(n, np.uint8)
    N.check(N.load().mh_verify_dual_proof_batch(_ctx(ctx).handle, C.byref(b), _addr(ok)))
    return ok.astype(bool)


def verify_dual_proof_v2_pb_batch(msgs, src, tgt, src_alh, tgt_alh,
                                  ctx: Optional[Context] = None) -> np.ndarray:
    """DualProofV2FromProto + VerifyDualProofV2 over many encoded DualProofV2
    messages in one device pass (mh_verify_dual_proof_v2_pb_batch) -> status[n]."""
    n = len(msgs)
    if n == 0:
        return np.zeros(0, np.int32)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in msgs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    s_, t_ = np.asarray(src, np.uint64), np.asarray(tgt, np.uint64)
    sa, ta = _d32(src_alh, n), _d32(tgt_alh, n)
    st = np.zeros(n, np.int32)
    N.check(N.load().mh_verify_dual_proof_v2_pb_batch(_ctx(ctx).handle, n, _addr(buf), _addr(off),
                                                      _addr(s_), _addr(t_), _addr(sa), _addr(ta),
                                                      _addr(st)))
    return st
