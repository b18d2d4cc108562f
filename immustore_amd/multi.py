"""Multi-GPU htree builds behind the C ABI (mh_multi_*).

One process drives K devices (the shape of a cgo caller: one Go process, the
commit path of immustore.go:1620-1632): one context (HIP stream) per device,
an RCCL clique over them inside libimmustore_merkle.so, power-of-two leaf
shards, one all-gather of the 32-byte subtree roots, the top levels reduced
on the devices.  bench.py's --gpus N path is the same decomposition with one
process per GPU over torch.distributed (immustore_amd/sharding.py).
"""
import ctypes as C
from typing import Sequence, Tuple

import numpy as np

from . import _native as N
from .merkle import _addr, levels_len


def shard_plan(n: int, ndev: int) -> Tuple[int, int]:
    """(S, G): shard size (power of two >= ceil(n / ndev)) and shard count."""
    s, g = C.c_uint64(), C.c_uint64()
    N.check(N.load().mh_multi_shard_plan(n, ndev, C.byref(s), C.byref(g)))
    return s.value, g.value


def ahtree_range_plan(n0: int, total: int, ndev: int) -> Tuple[int, list]:
    """(k, bounds): the ranges (bounds[d], bounds[d+1]] of a multi-device
    ahtree append of `total` appends onto a tree of n0 (interior bounds are
    multiples of 2^k), as mh_multi_(dev_)ahtree_append_batch cut them."""
    k, g = C.c_int(), C.c_int()
    b = (C.c_uint64 * (ndev + 1))()
    N.check(N.load().mh_ahtree_range_plan(n0, total, ndev, C.byref(k), b, C.byref(g)))
    return k.value, [b[i] for i in range(g.value + 1)]


def peaks_of(dlog: np.ndarray, n: int) -> bytes:
    """The popcount(n) peaks of a tree of size n (lowest level first) from a
    host dLog indexed from 0: node(n with the bits below l cleared, l)."""
    L = N.load()
    out = []
    for l in range(64):
        if (n >> l) & 1:
            out.append(bytes(dlog[L.mh_ahtree_node_index((n >> l) << l, l)]))
    return b"".join(out)


class MultiDevice:
    """mh_multi over the given device ordinals (a device may repeat: more
    shards than devices, roots gathered by device copies instead of RCCL)."""

    def __init__(self, devices: Sequence[int]):
        arr = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        N.check(N.load().mh_multi_create(len(devices), arr, C.byref(h)))
        self.handle = h.value
        self.devices = list(devices)

    def close(self):
        if self.handle:
            N.load().mh_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def uses_rccl(self) -> bool:
        """RCCL clique (distinct devices) vs device copies (a device repeats)."""
        return len(set(self.devices)) == len(self.devices)

    def ctx_handle(self, d: int):
        return N.load().mh_multi_ctx(self.handle, d)

    def synchronize(self):
        N.check(N.load().mh_multi_synchronize(self.handle))

    def build_entries_fixed(self, version: int, keys: np.ndarray, vals: np.ndarray,
                            want_levels: bool = True):
        """Host arrays keys (n, klen), vals (n, vlen) -> (hvals, levels, root)."""
        keys = np.ascontiguousarray(keys, np.uint8)
        vals = np.ascontiguousarray(vals, np.uint8)
        n = keys.shape[0]
        hv = np.zeros((max(n, 1), 32), np.uint8)
        lv = np.zeros((max(levels_len(n), 1), 32), np.uint8) if want_levels else None
        root = np.zeros(32, np.uint8)
        N.check(N.load().mh_multi_htree_build_entries_fixed(
            self.handle, version, n, _addr(keys), keys.shape[1], _addr(vals), vals.shape[1],
            _addr(hv), _addr(lv), _addr(root)))
        return hv[:n], (lv[:levels_len(n)] if want_levels else None), root.tobytes()

    def dev_build_entries_fixed(self, version, n_per_dev, keys, key_len, vals, val_len, levels,
                                top_levels, roots, hvals=None):
        """Device pointers per device (sequences of ints) -- asynchronous."""
        K = len(self.devices)
        P = C.c_void_p * K
        N.check(N.load().mh_multi_dev_htree_build_entries_fixed(
            self.handle, version, n_per_dev, P(*keys), key_len, P(*vals), val_len,
            P(*hvals) if hvals is not None else None, P(*levels), P(*top_levels), P(*roots)))

    def ahtree_append_batch(self, payloads, want_dlog: bool = True, n0: int = 0,
                            peaks: bytes = None):
        """AppendBatch of the rows of `payloads` (m, plen) onto an ahtree of
        size n0 with the given peaks (see peaks_of) across the devices ->
        (the NEW dLog digests (nodesUpto(n0+m) - nodesUpto(n0), 32) or None,
        RootAt(n0 + m))."""
        p = np.ascontiguousarray(payloads, np.uint8)
        m, plen = p.shape
        L = N.load()
        nd = L.mh_ahtree_nodes_upto(n0 + m) - L.mh_ahtree_nodes_upto(n0)
        dl = np.zeros((max(nd, 1), 32), np.uint8) if want_dlog else None
        root = np.zeros(32, np.uint8)
        pk = np.frombuffer(peaks, np.uint8) if peaks else None
        N.check(L.mh_multi_ahtree_append_batch(self.handle, n0, _addr(pk), _addr(p), m, plen,
                                                _addr(dl), _addr(root)))
        return (dl[:nd] if want_dlog else None), root.tobytes()

    def dev_ahtree_append_batch(self, total, payloads, plen, dlogs, roots_out=None, n0: int = 0,
                                peaks: bytes = None):
        """Device pointers per range (sequences of ints; None entries for
        unused ranges; range d as ahtree_range_plan cuts it) -- asynchronous."""
        K = len(self.devices)
        P = C.c_void_p * K
        pk = np.frombuffer(peaks, np.uint8) if peaks else None
        N.check(N.load().mh_multi_dev_ahtree_append_batch(
            self.handle, n0, _addr(pk), total, P(*payloads), plen, P(*dlogs),
            P(*roots_out) if roots_out is not None else None))

    def build_entries(self, version, kb, ko, mb, mo, vb, vo, ov=None, use=None,
                      want_levels: bool = True):
        """CSR host arrays (as mh_htree_build_entries; mb/mo and ov/use may be
        None) -> (hvals, levels, root)."""
        n = len(ko) - 1
        ko = np.ascontiguousarray(ko, np.uint64)
        vo = np.ascontiguousarray(vo, np.uint64)
        mo = None if mo is None else np.ascontiguousarray(mo, np.uint64)
        kb, vb = np.ascontiguousarray(kb, np.uint8), np.ascontiguousarray(vb, np.uint8)
        mb = None if mb is None else np.ascontiguousarray(mb, np.uint8)
        ov = None if ov is None else np.ascontiguousarray(ov, np.uint8)
        use = None if use is None else np.ascontiguousarray(use, np.uint8)
        hv = np.zeros((max(n, 1), 32), np.uint8)
        lv = np.zeros((max(levels_len(n), 1), 32), np.uint8) if want_levels else None
        root = np.zeros(32, np.uint8)
        N.check(N.load().mh_multi_htree_build_entries(
            self.handle, version, n, _addr(kb), _addr(ko), _addr(mb), _addr(mo), _addr(vb),
            _addr(vo), _addr(ov), _addr(use), _addr(hv), _addr(lv), _addr(root)))
        return hv[:n], (lv[:levels_len(n)] if want_levels else None), root.tobytes()

    # ---- the PCIe-bound batch paths split over the devices (mh_multi_*)
    def htree_verify_inclusion_batch(self, leaf, width, term_off, terms, digests, roots):
        """Raw arrays as mh_htree_verify_inclusion_batch (leaf / width uint64
        Go-int patterns, CSR term_off, terms (T, 32), digests / roots (n, 32))
        -> ok[n] bool; proofs split by index over the devices."""
        leaf = np.ascontiguousarray(leaf, np.uint64)
        width = np.ascontiguousarray(width, np.uint64)
        off = np.ascontiguousarray(term_off, np.uint64)
        terms = np.ascontiguousarray(terms, np.uint8).reshape(-1, 32)
        if terms.size == 0:
            terms = np.zeros((1, 32), np.uint8)
        d = np.ascontiguousarray(digests, np.uint8)
        r = np.ascontiguousarray(roots, np.uint8)
        n = leaf.size
        ok = np.zeros(max(n, 1), np.uint8)
        N.check(N.load().mh_multi_htree_verify_inclusion_batch(
            self.handle, n, _addr(leaf), _addr(width), _addr(off), _addr(terms), _addr(d), _addr(r),
            _addr(ok)))
        return ok[:n].astype(bool)

    def verify_dual_proof_v2_batch(self, src_hdrs, tgt_hdrs, md_blob, incl, cons, src, tgt,
                                   src_alh, tgt_alh):
        """txlayer.verify_dual_proof_v2_batch's arguments -> status[n]; split
        by index over the devices."""
        from .txlayer import _blob, _d32, _hdrs, _terms_csr
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
        N.check(N.load().mh_multi_verify_dual_proof_v2_batch(
            self.handle, n, _addr(sh), _addr(th), _addr(mb), ml, _addr(io), _addr(it), _addr(co),
            _addr(ct), _addr(s), _addr(t), _addr(sa), _addr(ta), _addr(st)))
        return st

    def verify_values(self, vals, off, hvals, vlen=None):
        """merkle.verify_values over the devices (mh_multi_verify_values_batch:
        parts of nearly equal value bytes) -> (corrupted count, status[n])."""
        off = np.ascontiguousarray(off, np.uint64)
        n = len(off) - 1
        v = np.ascontiguousarray(vals, np.uint8)
        hv = np.ascontiguousarray(hvals, np.uint8)
        vl = None if vlen is None else np.ascontiguousarray(vlen, np.uint64)
        st = np.zeros(max(n, 1), np.int32)
        bad = C.c_uint64()
        N.check(N.load().mh_multi_verify_values_batch(
            self.handle, n, _addr(v) if v.size else None, _addr(off), _addr(vl), _addr(hv),
            _addr(st), C.byref(bad)))
        return bad.value, st[:n]

    def verify_dual_proof_v2_pb_batch(self, msgs, src, tgt, src_alh, tgt_alh):
        """txlayer.verify_dual_proof_v2_pb_batch over the devices (parts of
        nearly equal message bytes) -> status[n]."""
        from .txlayer import _d32
        n = len(msgs)
        if n == 0:
            return np.zeros(0, np.int32)
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in msgs], dtype=np.uint64)
        buf = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
        s_, t_ = np.asarray(src, np.uint64), np.asarray(tgt, np.uint64)
        sa, ta = _d32(src_alh, n), _d32(tgt_alh, n)
        st = np.zeros(n, np.int32)
        N.check(N.load().mh_multi_verify_dual_proof_v2_pb_batch(
            self.handle, n, _addr(buf), _addr(off), _addr(s_), _addr(t_), _addr(sa), _addr(ta),
            _addr(st)))
        return st

    def verify_document_batch(self, docs):
        """txlayer.verify_document_batch over the devices
        (mh_multi_verify_document_batch) -> (status[n], target_alh[n, 32])."""
        from .txlayer import pack_document_batch
        n = len(docs)
        if n == 0:
            return np.zeros(0, np.int32), np.zeros((0, 32), np.uint8)
        b, keep = pack_document_batch(docs)
        st = np.zeros(n, np.int32)
        alh = np.zeros((n, 32), np.uint8)
        N.check(N.load().mh_multi_verify_document_batch(self.handle, C.byref(b), _addr(st),
                                                        _addr(alh)))
        del keep
        return st, alh

    def precommit_csr(self, version: int, tx_off, keys, key_off, vals, val_off, md=None,
                      md_off=None, hval_override=None, use_override=None, expect_eh=None,
                      max_width: int = 0):
        """commit.CommitPipe.precommit_csr over the devices
        (mh_multi_precommit_batch: whole transactions, parts of nearly equal
        value bytes, a commit pipe per device) -> (hvals, eh, status)."""
        tx_off = np.ascontiguousarray(tx_off, np.uint64)
        ntx = len(tx_off) - 1
        ne = int(tx_off[-1] - tx_off[0]) if ntx > 0 else 0
        hv = np.zeros((max(ne, 1), 32), np.uint8)
        eh = np.zeros((max(ntx, 1), 32), np.uint8)
        st = np.zeros(max(ntx, 1), np.int32)
        N.check(N.load().mh_multi_precommit_batch(
            self.handle, version, max_width, ntx, _addr(tx_off), _addr(keys), _addr(key_off),
            _addr(md), _addr(md_off), _addr(vals), _addr(val_off), _addr(hval_override),
            _addr(use_override), _addr(expect_eh), _addr(hv), _addr(eh), _addr(st)))
        return hv[:ne], eh[:ntx], st[:ntx]

    def txlog_validate(self, buf, max_entries: int = 1024, max_key_len: int = 1024,
                       max_txs=None, out=None):
        """txlayer.txlog_validate over the devices (mh_multi_txlog_validate:
        the log cut at record boundaries, every part over its own link) ->
        (status, ntx, consumed, hdrs, alh, per_tx)."""
        from .txlayer import TX_HEADER
        b = np.frombuffer(bytes(buf), np.uint8) if not isinstance(buf, np.ndarray) else buf
        cap = max(1, b.size // 122 + 1)
        if max_txs is not None:
            cap = max(1, min(cap, max_txs))
        if out is not None:
            hd, alh, sts = out
            cap = max(1, min(cap, len(alh), len(sts), len(hd) if hd is not None else cap))
        else:
            hd = np.empty(cap, TX_HEADER)
            alh = np.empty((cap, 32), np.uint8)
            sts = np.empty(cap, np.int32)
        ntx, used = C.c_uint64(0), C.c_uint64(0)
        rc = N.load().mh_multi_txlog_validate(self.handle, _addr(b) if b.size else None, b.size,
                                              max_entries, max_key_len, cap, C.byref(ntx),
                                              C.byref(used), _addr(hd) if hd is not None else None,
                                              _addr(alh), _addr(sts))
        if rc < 0:
            N.check(rc)
        k = ntx.value
        return rc, k, used.value, (hd[:k] if hd is not None else None), alh[:k], sts[:k]
