"""ctypes binding of oracle/liboracle.so -- the CPU restatement of the path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
`cpu_baseline` leg of bench.py, always as the checker / baseline, never as the
thing measured or shipped.  immustore_amd/ never imports this module.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_KEEP = []

u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)


def _p(a, t=u8p):
    if a is None:
        return None
    return a.ctypes.data_as(t)


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_sha256.argtypes = [u8p, C.c_size_t, u8p]
        L.orc_entry_digest.argtypes = [C.c_int, u8p, C.c_size_t, u8p, C.c_size_t, u8p, u8p]
        L.orc_htree_levels_len.restype = C.c_uint64
        L.orc_htree_levels_len.argtypes = [C.c_uint64]
        L.orc_htree_level_offset.restype = C.c_uint64
        L.orc_htree_level_offset.argtypes = [C.c_uint64, C.c_int]
        L.orc_htree_build.argtypes = [u8p, C.c_uint64, u8p, u8p]
        L.orc_htree_inclusion_proof.argtypes = [u8p, C.c_uint64, C.c_uint64, u8p, u32p]
        L.orc_htree_verify_inclusion.argtypes = [C.c_uint64, C.c_uint64, u8p, C.c_uint32, u8p, u8p]
        L.orc_build_entries.argtypes = [C.c_int, C.c_uint64, u8p, u64p, u8p, u64p, u8p, u64p,
                                        u8p, u8p, u8p, u8p, u8p]
        L.orc_build_entries_fixed.argtypes = [C.c_int, C.c_uint64, u8p, C.c_uint32, u8p,
                                              C.c_uint32, u8p, u8p, u8p, C.c_int]
        L.orc_tx_inner_hash.argtypes = [C.c_uint64, C.c_int, u8p, C.c_size_t, C.c_uint32, u8p,
                                        C.c_uint64, u8p, u8p]
        L.orc_tx_alh.argtypes = [C.c_uint64, u8p, u8p, u8p]
        L.orc_ahtree_nodes_upto.restype = C.c_uint64
        L.orc_ahtree_nodes_upto.argtypes = [C.c_uint64]
        L.orc_ahtree_nodes_until.restype = C.c_uint64
        L.orc_ahtree_nodes_until.argtypes = [C.c_uint64]
        L.orc_ahtree_append.argtypes = [u8p, C.c_uint64, u8p, C.c_size_t, u8p]
        L.orc_ahtree_append_batch.argtypes = [u8p, C.c_uint64, u8p, C.c_uint64, C.c_size_t]
        L.orc_ahtree_log_records.argtypes = [u8p, C.c_uint64, C.c_size_t, C.c_uint64, u8p, u8p]
        L.orc_ahtree_log_records.restype = None
        L.orc_ahtree_root_at.argtypes = [u8p, C.c_uint64, C.c_uint64, u8p]
        L.orc_ahtree_inclusion_proof.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint64, u8p, u32p]
        L.orc_ahtree_consistency_proof.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint64, u8p, u32p]
        L.orc_ahtree_eval_inclusion.argtypes = [u8p, C.c_uint32, C.c_uint64, C.c_uint64, u8p, u8p]
        L.orc_ahtree_verify_inclusion.argtypes = [u8p, C.c_uint32, C.c_uint64, C.c_uint64, u8p, u8p]
        L.orc_ahtree_eval_consistency.argtypes = [u8p, C.c_uint32, C.c_uint64, C.c_uint64, u8p, u8p]
        L.orc_ahtree_verify_consistency.argtypes = [u8p, C.c_uint32, C.c_uint64, C.c_uint64, u8p, u8p]
        L.orc_ahtree_eval_last_inclusion.argtypes = [u8p, C.c_uint32, C.c_uint64, u8p, u8p]
        L.orc_ahtree_verify_last_inclusion.argtypes = [u8p, C.c_uint32, C.c_uint64, u8p, u8p]
        L.orc_fill_random.argtypes = [u8p, C.c_uint64, C.c_uint64]
        L.orc_tx_header_alh.argtypes = [u8p, u8p, u8p, u8p]
        L.orc_htree_verify_batch.restype = C.c_uint64
        L.orc_htree_verify_batch.argtypes = [C.c_uint64, u64p, C.c_uint64, u8p, C.c_uint32, u8p,
                                             u8p, u8p]
        L.orc_ahtree_verify_batch.restype = C.c_uint64
        L.orc_ahtree_verify_batch.argtypes = [C.c_int, C.c_uint64, u64p, u64p, u64p, u8p, u8p,
                                              u8p, u8p, C.c_int]
        L.orc_verify_linear_proof.argtypes = [C.c_uint64, C.c_uint64, u8p, C.c_uint32, C.c_uint64,
                                              C.c_uint64, u8p, u8p]
        L.orc_verify_linear_advance_proof.argtypes = [C.c_int, u8p, C.c_uint32, u8p, u32p,
                                                      C.c_uint32, C.c_uint64, C.c_uint64, u8p,
                                                      u8p, C.c_uint64]
        L.orc_verify_dual_proof_v2.argtypes = [u8p, u8p, u8p, u8p, C.c_uint32, u8p, C.c_uint32,
                                               C.c_uint64, C.c_uint64, u8p, u8p]
        L.orc_verify_dual_proof.argtypes = [u8p, u8p, u8p, u8p, C.c_uint32, u8p, C.c_uint32, u8p,
                                            u8p, C.c_uint32, C.c_int, C.c_uint64, C.c_uint64, u8p,
                                            C.c_uint32, C.c_int, u8p, C.c_uint32, u8p, u32p,
                                            C.c_uint32, C.c_uint64, C.c_uint64, u8p, u8p]
        L.orc_txlog_validate.argtypes = [u8p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64,
                                         u64p, u64p, u8p, C.POINTER(C.c_int32)]
        L.orc_sha256_use_shani.argtypes = [C.c_int]
        L.orc_ahtree_proof_batch.argtypes = [u8p, C.c_uint64, C.c_int, C.c_uint64, u64p, u64p,
                                             u8p, C.c_uint32, u32p, C.POINTER(C.c_int32)]
        L.orc_ahtree_proof_batch.restype = None
        L.orc_ahtree_stream.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, u8p,
                                        C.c_uint64, u64p, C.c_uint64, u8p, u32p, u8p]
        L.orc_precommit_batch.argtypes = [C.c_int, C.c_uint64, C.c_uint64, u64p, u8p, u64p, u8p,
                                          u64p, u8p, u64p, u8p, u8p, u8p, u8p, u8p,
                                          C.POINTER(C.c_int32), C.c_int]
        _LIB = L
    return _LIB


def _u8(b):
    return np.frombuffer(bytes(b), dtype=np.uint8).copy() if not isinstance(b, np.ndarray) else b


def sha256(b):
    a = _u8(b)
    out = np.zeros(32, np.uint8)
    lib().orc_sha256(_p(a) if len(a) else None, len(a), _p(out))
    return out.tobytes()


def entry_digest(version, key, md, hval):
    k, m, h = _u8(key), _u8(md), _u8(hval)
    out = np.zeros(32, np.uint8)
    st = lib().orc_entry_digest(version, _p(k) if len(k) else None, len(k),
                                _p(m) if len(m) else None, len(m), _p(h), _p(out))
    return st, out.tobytes()


def levels_len(n):
    return lib().orc_htree_levels_len(n)


def level_offset(n, l):
    return lib().orc_htree_level_offset(n, l)


def htree_build(digests):
    """digests: (n,32) uint8 -> (levels flat (L,32), root bytes)."""
    d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1, 32)
    n = d.shape[0]
    lv = np.zeros((max(levels_len(n), 1), 32), np.uint8)
    root = np.zeros(32, np.uint8)
    lib().orc_htree_build(_p(d) if n else None, n, _p(lv), _p(root))
    return lv[:levels_len(n)], root.tobytes()


def htree_inclusion_proof(levels, width, i):
    terms = np.zeros((64, 32), np.uint8)
    nt = C.c_uint32(0)
    st = lib().orc_htree_inclusion_proof(_p(np.ascontiguousarray(levels)), width, i, _p(terms),
                                         C.byref(nt))
    return st, terms[:nt.value].copy()


def htree_verify_inclusion(leaf, width, terms, digest, root):
    tp, nt = _terms(terms)
    return bool(lib().orc_htree_verify_inclusion(leaf, width, tp, nt, _p(_u8(digest)),
                                                 _p(_u8(root))))


def build_entries_fixed(version, keys, vals, nthreads=1, want_levels=True):
    """keys (n,klen) u8, vals (n,vlen) u8 -> (hvals, levels, root)."""
    n = keys.shape[0]
    hv = np.zeros((n, 32), np.uint8)
    lv = np.zeros((max(levels_len(n), 1), 32), np.uint8) if want_levels else None
    root = np.zeros(32, np.uint8)
    st = lib().orc_build_entries_fixed(version, n, _p(keys), keys.shape[1], _p(vals), vals.shape[1],
                                       _p(hv), _p(lv), _p(root), nthreads)
    assert st == 0, st
    return hv, (lv[:levels_len(n)] if want_levels else None), root.tobytes()


def build_entries(version, keys, mds, vals, overrides=None):
    """Lists of bytes -> (status, hvals, levels, root)."""
    n = len(keys)

    def csr(items):
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in items]) if n else []
        buf = np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8).copy()
        return buf, off

    kb, ko = csr(keys)
    mb, mo = csr(mds)
    vb, vo = csr(vals)
    ov = use = None
    if overrides is not None:
        ov = np.zeros((n, 32), np.uint8)
        use = np.zeros(n, np.uint8)
        for i, o in enumerate(overrides):
            if o is not None:
                ov[i] = np.frombuffer(o, np.uint8)
                use[i] = 1
    hv = np.zeros((max(n, 1), 32), np.uint8)
    lv = np.zeros((max(levels_len(n), 1), 32), np.uint8)
    root = np.zeros(32, np.uint8)
    st = lib().orc_build_entries(version, n, _p(kb), _p(ko, u64p), _p(mb), _p(mo, u64p), _p(vb),
                                 _p(vo, u64p), _p(ov), _p(use), _p(hv), _p(lv), _p(root))
    return st, hv[:n], lv[:levels_len(n)], root.tobytes()


def build_entries_csr(version, kb, ko, mb, mo, vb, vo, want_levels=True, ov=None, use=None):
    """CSR byte arrays (u8) + u64 offsets (n+1 each; mb/mo may be None) ->
    (status, hvals, levels, root); the array form of build_entries for large
    ragged batches.  ov (n x 32) / use (n, u8): IsValueTruncated hVal
    overrides."""
    n = len(ko) - 1
    ko, vo = np.ascontiguousarray(ko, np.uint64), np.ascontiguousarray(vo, np.uint64)
    mo = None if mo is None else np.ascontiguousarray(mo, np.uint64)
    hv = np.zeros((max(n, 1), 32), np.uint8)
    lv = np.zeros((max(levels_len(n), 1), 32), np.uint8) if want_levels else None
    root = np.zeros(32, np.uint8)
    ov = None if ov is None else np.ascontiguousarray(ov, np.uint8)
    use = None if use is None else np.ascontiguousarray(use, np.uint8)
    st = lib().orc_build_entries(version, n, _p(kb), _p(ko, u64p), _p(mb), _p(mo, u64p), _p(vb),
                                 _p(vo, u64p), _p(ov), _p(use), _p(hv), _p(lv), _p(root))
    return st, hv[:n], (lv[:levels_len(n)] if want_levels else None), root.tobytes()


def precommit_batch(version, tx_off, keys, key_off, vals, val_off, md=None, md_off=None,
                    hval_override=None, use_override=None, expect_eh=None, max_width=0,
                    nthreads=1):
    """ImmuStore.precommit over many txs (immustore.go:1620-1632, :1649-1654), CSR
    numpy inputs as for mh_precommit_batch -> (hvals [E,32], eh [ntx,32], status)."""
    ntx = len(tx_off) - 1
    ne = int(tx_off[-1] - tx_off[0]) if ntx > 0 else 0
    hv = np.zeros((max(ne, 1), 32), np.uint8)
    eh = np.zeros((max(ntx, 1), 32), np.uint8)
    st = np.zeros(max(ntx, 1), np.int32)
    tx_off = np.ascontiguousarray(tx_off, np.uint64)
    lib().orc_precommit_batch(version, max_width, ntx, _p(tx_off, u64p), _p(keys),
                              _p(key_off, u64p), _p(md), _p(md_off, u64p), _p(vals),
                              _p(val_off, u64p), _p(hval_override), _p(use_override),
                              _p(expect_eh), _p(hv), _p(eh),
                              st.ctypes.data_as(C.POINTER(C.c_int32)), nthreads)
    return hv[:ne], eh[:ntx], st[:ntx]


def tx_inner_hash(ts, version, txmd, nentries, eh, bltxid, blroot):
    m = _u8(txmd)
    out = np.zeros(32, np.uint8)
    st = lib().orc_tx_inner_hash(ts, version, _p(m) if len(m) else None, len(m), nentries,
                                 _p(_u8(eh)), bltxid, _p(_u8(blroot)), _p(out))
    return st, out.tobytes()


def tx_alh(txid, prev_alh, inner):
    out = np.zeros(32, np.uint8)
    lib().orc_tx_alh(txid, _p(_u8(prev_alh)), _p(_u8(inner)), _p(out))
    return out.tobytes()


def nodes_upto(n):
    return lib().orc_ahtree_nodes_upto(n)


def nodes_until(n):
    return lib().orc_ahtree_nodes_until(n)


class AHtree:
    """Growable in-memory dLog over the oracle's ahtree functions."""

    def __init__(self, cap=1024):
        self.size = 0
        self.dlog = np.zeros((nodes_upto(cap), 32), np.uint8)

    def _grow(self, n):
        need = nodes_upto(n)
        if need > self.dlog.shape[0]:
            nd = np.zeros((max(need, 2 * self.dlog.shape[0]), 32), np.uint8)
            nd[:self.dlog.shape[0]] = self.dlog
            self.dlog = nd

    def append(self, payload):
        p = _u8(payload)
        self._grow(self.size + 1)
        r = np.zeros(32, np.uint8)
        lib().orc_ahtree_append(_p(self.dlog), self.size, _p(p) if len(p) else None, len(p), _p(r))
        self.size += 1
        return r.tobytes()

    def append_batch(self, payloads):
        p = np.ascontiguousarray(payloads, np.uint8)
        m, plen = p.shape
        self._grow(self.size + m)
        lib().orc_ahtree_append_batch(_p(self.dlog), self.size, _p(p), m, plen)
        self.size += m

    def append_batch_logs(self, payloads, p_off0):
        """append_batch plus the pLog / cLog record streams of the batch
        (ahtree.go:266-282, 341-351) -> (plog bytes, clog bytes)."""
        p = np.ascontiguousarray(payloads, np.uint8)
        m, plen = p.shape
        plog = np.zeros(max(1, m * (4 + plen)), np.uint8)
        clog = np.zeros(max(1, m * 12), np.uint8)
        lib().orc_ahtree_log_records(_p(p), m, plen, p_off0, _p(plog), _p(clog))
        self.append_batch(p)
        return plog[:m * (4 + plen)].tobytes(), clog[:m * 12].tobytes()

    def dlog_bytes(self):
        return self.dlog[:nodes_upto(self.size)].tobytes()

    def root_at(self, n):
        out = np.zeros(32, np.uint8)
        st = lib().orc_ahtree_root_at(_p(self.dlog), self.size, n, _p(out))
        return st, out.tobytes()

    def inclusion_proof(self, i, j):
        t = np.zeros((192, 32), np.uint8)
        nt = C.c_uint32(0)
        st = lib().orc_ahtree_inclusion_proof(_p(self.dlog), self.size, i, j, _p(t), C.byref(nt))
        return st, t[:nt.value].copy()

    def consistency_proof(self, i, j):
        t = np.zeros((192, 32), np.uint8)
        nt = C.c_uint32(0)
        st = lib().orc_ahtree_consistency_proof(_p(self.dlog), self.size, i, j, _p(t), C.byref(nt))
        return st, t[:nt.value].copy()

    def proof_batch(self, kind, i, j, cap=64):
        """kind 0 / 1: InclusionProof / ConsistencyProof for every (i[p], j[p])
        -> (terms (n, cap, 32), nterms (n,), status (n,))."""
        i = np.ascontiguousarray(i, np.uint64)
        j = np.ascontiguousarray(j, np.uint64)
        n = len(i)
        t = np.zeros((max(n, 1), cap, 32), np.uint8)
        nt = np.zeros(max(n, 1), np.uint32)
        st = np.zeros(max(n, 1), np.int32)
        lib().orc_ahtree_proof_batch(_p(self.dlog), self.size, kind, n, _p(i, u64p), _p(j, u64p),
                                     _p(t), cap, _p(nt, u32p), st.ctypes.data_as(C.POINTER(C.c_int32)))
        return t[:n], nt[:n], st[:n]


def _terms(t):
    if not isinstance(t, np.ndarray):
        t = np.frombuffer(b"".join(bytes(x) for x in t), dtype=np.uint8) if len(t) else \
            np.zeros((0, 32), np.uint8)
    t = np.ascontiguousarray(t, dtype=np.uint8).reshape(-1, 32)
    _KEEP.append(t)  # keep alive until the call returns
    if len(_KEEP) > 64:
        del _KEEP[:32]
    return (_p(t) if len(t) else None), len(t)


def ahtree_verify_inclusion(proof, i, j, leaf, root):
    tp, nt = _terms(proof)
    return bool(lib().orc_ahtree_verify_inclusion(tp, nt, i, j, _p(_u8(leaf)), _p(_u8(root))))


def ahtree_eval_inclusion(proof, i, j, leaf):
    tp, nt = _terms(proof)
    out = np.zeros(32, np.uint8)
    lib().orc_ahtree_eval_inclusion(tp, nt, i, j, _p(_u8(leaf)), _p(out))
    return out.tobytes()


def ahtree_verify_consistency(proof, i, j, iroot, jroot):
    tp, nt = _terms(proof)
    return bool(lib().orc_ahtree_verify_consistency(tp, nt, i, j, _p(_u8(iroot)), _p(_u8(jroot))))


def ahtree_eval_consistency(proof, i, j):
    tp, nt = _terms(proof)
    ci = np.zeros(32, np.uint8)
    cj = np.zeros(32, np.uint8)
    st = lib().orc_ahtree_eval_consistency(tp, nt, i, j, _p(ci), _p(cj))
    return st, ci.tobytes(), cj.tobytes()


def ahtree_verify_last_inclusion(proof, i, leaf, root):
    tp, nt = _terms(proof)
    return bool(lib().orc_ahtree_verify_last_inclusion(tp, nt, i, _p(_u8(leaf)), _p(_u8(root))))


def verify_values(vals, off, hvals, vlen=None, nthreads=1):
    """readValueAt's check (immustore.go:3235) per value -> (bad count,
    status int32[n]: 0 or 14 = ErrCorruptedData)."""
    off = np.ascontiguousarray(off, np.uint64)
    n = len(off) - 1
    v = np.ascontiguousarray(vals, np.uint8)
    if v.size == 0:
        v = np.zeros(1, np.uint8)
    hv = np.ascontiguousarray(hvals, np.uint8)
    vl = None if vlen is None else np.ascontiguousarray(vlen, np.uint64)
    st = np.zeros(max(n, 1), np.int32)
    L = lib()
    L.orc_verify_values.restype = C.c_uint64
    bad = L.orc_verify_values(C.c_uint64(n), _p(v), _p(off), _p(vl) if vl is not None else None,
                              _p(hv), st.ctypes.data_as(C.c_void_p), nthreads)
    return int(bad), st[:n]


def fill_random(nbytes, seed):
    out = np.zeros(nbytes, np.uint8)
    lib().orc_fill_random(_p(out), nbytes, seed)
    return out


def ahtree_stream(seed, plen, n_start, n_end, samples=(), peaks_in=None, pay0=None):
    """orc_ahtree_stream: appends (n_start, n_end] of fill_random(seed)
    payloads (append n takes payload pay0 + n - n_start - 1; pay0 defaults to
    n_start, i.e. payload n-1 of the one stream) kept as peaks only ->
    ({n: [digests append n writes to the dLog]}, peaks of n_end as a (64, 32)
    array, slot l meaningful for set bits l of n_end)."""
    L = lib()
    s = np.ascontiguousarray(sorted(set(int(x) for x in samples)), np.uint64)
    out = np.zeros((max(len(s), 1), 65, 32), np.uint8)
    cnt = np.zeros(max(len(s), 1), np.uint32)
    pk = np.zeros((64, 32), np.uint8)
    pin = None if peaks_in is None else np.ascontiguousarray(peaks_in, np.uint8).reshape(64, 32)
    st = L.orc_ahtree_stream(seed, plen, n_start if pay0 is None else pay0, n_start,
                             _p(pin) if pin is not None else None, n_end,
                             _p(s, u64p) if len(s) else None, len(s), _p(out), _p(cnt, u32p),
                             _p(pk))
    if st:
        raise ValueError("orc_ahtree_stream: status %d" % st)
    return {int(n): [bytes(out[i, c]) for c in range(cnt[i])] for i, n in enumerate(s)}, pk


def ahtree_peaks_streamed(seed, plen, n, threads=1, block_bits=20):
    """The peaks of a tree of n appends of fill_random(seed) payloads, as a
    (64, 32) array, without its dLog: peak l (set bit l of n) is the perfect
    subtree over the aligned block of 2^l appends ending at n with the bits
    below l cleared (ahtree.go:460-462); a block of 2^l payloads is the root
    of the perfect tree over them alone, so every block is cut into
    sub-blocks of <= 2^block_bits payloads streamed on `threads` host threads
    (orc_ahtree_stream, GIL released) and their roots paired
    SHA256(0x01 || left || right) up to level l."""
    from concurrent.futures import ThreadPoolExecutor
    jobs = []  # (level, first payload, sub-block bits)
    for l in range(64):
        if (n >> l) & 1:
            a = (n >> (l + 1)) << (l + 1)
            sb = min(l, block_bits)
            for j in range(1 << (l - sb)):
                jobs.append((l, a + (j << sb), sb))

    def root_of(job):
        _, first, sb = job
        _, pk = ahtree_stream(seed, plen, 0, 1 << sb, pay0=first)
        return bytes(pk[sb])

    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        roots = list(ex.map(root_of, jobs))
    out = np.zeros((64, 32), np.uint8)
    k = 0
    for l in range(64):
        if (n >> l) & 1:
            sb = min(l, block_bits)
            row = roots[k:k + (1 << (l - sb))]
            k += len(row)
            while len(row) > 1:
                row = [sha256(b"\x01" + row[i] + row[i + 1]) for i in range(0, len(row), 2)]
            out[l] = np.frombuffer(row[0], np.uint8)
    return out


def use_shani(enable):
    lib().orc_sha256_use_shani(1 if enable else 0)


def has_shani():
    return bool(lib().orc_sha256_has_shani())


# ---------------------------------------------------------------- tx layer
# Same layout as orc_tx_header / include/immustore_merkle.h mh_tx_header.
TX_HEADER = np.dtype([("id", "<u8"), ("ts", "<i8"), ("bl_tx_id", "<u8"), ("bl_root", "u1", 32),
                      ("prev_alh", "u1", 32), ("eh", "u1", 32), ("version", "<u4"),
                      ("nentries", "<u4"), ("md_len", "<u4"), ("md_off", "<u4")])
assert TX_HEADER.itemsize == 136


def tx_header_alh(hdr, md_blob=b""):
    """hdr: a TX_HEADER record (np.void or 1-element array)."""
    h = np.ascontiguousarray(np.asarray(hdr, TX_HEADER).reshape(1))
    mb = _u8(md_blob) if len(md_blob) else np.zeros(1, np.uint8)
    inner, alh = np.zeros(32, np.uint8), np.zeros(32, np.uint8)
    st = lib().orc_tx_header_alh(_p(h.view(np.uint8)), _p(mb), _p(inner), _p(alh))
    return st, inner.tobytes(), alh.tobytes()


def verify_linear_proof(p_src, p_tgt, terms, src, tgt, src_alh, tgt_alh):
    tp, nt = _terms(terms)
    return bool(lib().orc_verify_linear_proof(p_src, p_tgt, tp, nt, src, tgt,
                                              _p(_u8(src_alh)), _p(_u8(tgt_alh))))


def verify_linear_advance_proof(proof, start, end, end_alh, root, size):
    """proof: None or (linear_terms, [inclusion_terms, ...])."""
    if proof is None:
        z = np.zeros((1, 32), np.uint8)
        return bool(lib().orc_verify_linear_advance_proof(0, _p(z), 0, _p(z), None, 0, start, end,
                                                          _p(_u8(end_alh)), _p(_u8(root)), size))
    lin, incs = proof
    lp, nl = _terms(lin)
    off = np.zeros(len(incs) + 1, np.uint32)
    for k, ip in enumerate(incs):
        off[k + 1] = off[k] + len(ip)
    ip_, _ = _terms([x for ip in incs for x in ip])
    return bool(lib().orc_verify_linear_advance_proof(1, lp, nl, ip_, _p(off, u32p), len(incs),
                                                      start, end, _p(_u8(end_alh)),
                                                      _p(_u8(root)), size))


def verify_dual_proof_v2(sh, th, md_blob, incl, cons, src, tgt, src_alh, tgt_alh):
    a = np.ascontiguousarray(np.asarray(sh, TX_HEADER).reshape(1))
    b = np.ascontiguousarray(np.asarray(th, TX_HEADER).reshape(1))
    mb = _u8(md_blob) if len(md_blob) else np.zeros(1, np.uint8)
    ip_, ni = _terms(incl)
    cp_, nc = _terms(cons)
    return lib().orc_verify_dual_proof_v2(_p(a.view(np.uint8)), _p(b.view(np.uint8)), _p(mb),
                                          ip_, ni, cp_, nc, src, tgt,
                                          _p(_u8(src_alh)), _p(_u8(tgt_alh)))


def txlog_validate(buf, max_entries=1024, max_key_len=1024, max_txs=1 << 40):
    """-> (status, ntx, consumed, alh[ntx,32], per_tx_status[ntx])"""
    b = _u8(buf) if len(buf) else np.zeros(1, np.uint8)
    cap = max(1, min(max_txs, len(buf) // 90 + 1))
    alh = np.zeros((cap, 32), np.uint8)
    sts = np.zeros(cap, np.int32)
    ntx, used = C.c_uint64(0), C.c_uint64(0)
    st = lib().orc_txlog_validate(_p(b), len(buf), max_entries, max_key_len, min(max_txs, cap),
                                  C.byref(ntx), C.byref(used), _p(alh),
                                  sts.ctypes.data_as(C.POINTER(C.c_int32)))
    n = ntx.value
    return st, n, used.value, alh[:n].copy(), sts[:n].copy()


ERR_CORRUPTED_DATA = 14
ERR_TRUNCATED = 18


def txlog_validate_clog(buf, clog, es=12, max_entries=1024, max_key_len=1024):
    """ImmuStore.readTx (embedded/store/immustore.go:3048-3060) of txs 1..n
    located by the commit-log entries clog (txOffsetAndSize, :2569-2597: BE64
    offset || BE32 size [|| Alh], es = 12 or 44 bytes, :122-123), each read from
    its offset on to the end of the log (the reader is not bounded by the
    size), plus the open path's cLog checks (:458-528: the record ends at
    offset + size; a 44-byte entry's Alh is the tx's).
    -> (alh[n,32], status[n]); alh is zero where the record's structure or the
    cLog checks fail (status: the reader's error, MH_ERR_TRUNCATED for its
    unexpected EOF, MH_ERR_CORRUPTED_DATA for a cLog mismatch)."""
    import struct
    b = _u8(buf) if len(buf) else np.zeros(1, np.uint8)
    blen = len(buf)
    n = len(clog) // es
    alh = np.zeros((n, 32), np.uint8)
    sts = np.zeros(n, np.int32)
    one_a = np.zeros((1, 32), np.uint8)
    one_s = np.zeros(1, np.int32)
    base = b.ctypes.data
    for t in range(n):
        off, size = struct.unpack_from(">QI", clog, t * es)
        if off + 8 > blen:
            sts[t] = ERR_TRUNCATED
            continue
        ntx, used = C.c_uint64(0), C.c_uint64(0)
        st = lib().orc_txlog_validate(C.cast(base + off, u8p), blen - off, max_entries, max_key_len,
                                      1, C.byref(ntx), C.byref(used), _p(one_a),
                                      one_s.ctypes.data_as(C.POINTER(C.c_int32)))
        if st == 0 and ntx.value == 0:
            st = ERR_TRUNCATED  # an id-0 record: the reader's EOF
        if st == 0 and used.value != size:
            st = ERR_CORRUPTED_DATA
        if st == 0 and es == 44 and bytes(clog[t * es + 12:t * es + 44]) != \
                b[off + size - 32:off + size].tobytes():
            st = ERR_CORRUPTED_DATA
        if st == 0:
            sts[t] = one_s[0]
            alh[t] = one_a[0]
        else:
            sts[t] = st
    return alh, sts


def verify_dual_proof(sh, th, md_blob, incl, cons, tbl_alh, last, lin, lap, src, tgt, src_alh,
                      tgt_alh):
    """VerifyDualProof (v1).  lin: None or (lin_src, lin_tgt, terms); lap: None or
    (linear_terms, [inclusion_terms, ...])."""
    a = np.ascontiguousarray(np.asarray(sh, TX_HEADER).reshape(1))
    b = np.ascontiguousarray(np.asarray(th, TX_HEADER).reshape(1))
    mb = _u8(md_blob) if len(md_blob) else np.zeros(1, np.uint8)
    ip_, ni = _terms(incl)
    cp_, nc = _terms(cons)
    lp_, nl = _terms(last)
    if lin is None:
        has_lin, ls, lt, lin_p, nlin = 0, 0, 0, None, 0
    else:
        has_lin, (ls, lt, lterms) = 1, lin
        lin_p, nlin = _terms(lterms)
    if lap is None:
        has_lap, lap_p, nlap, inc_p, off, ninc = 0, None, 0, None, np.zeros(1, np.uint32), 0
    else:
        has_lap = 1
        lap_p, nlap = _terms(lap[0])
        off = np.zeros(len(lap[1]) + 1, np.uint32)
        for k, ip in enumerate(lap[1]):
            off[k + 1] = off[k] + len(ip)
        inc_p, _ = _terms([x for ip in lap[1] for x in ip])
        ninc = len(lap[1])
    return bool(lib().orc_verify_dual_proof(
        _p(a.view(np.uint8)), _p(b.view(np.uint8)), _p(mb), ip_, ni, cp_, nc, _p(_u8(tbl_alh)),
        lp_, nl, has_lin, ls, lt, lin_p, nlin, has_lap, lap_p, nlap, inc_p, _p(off, u32p), ninc,
        src, tgt, _p(_u8(src_alh)), _p(_u8(tgt_alh))))


def htree_verify_batch(leaf, width, terms, digests, root):
    """terms: (n, D, 32) uint8; returns (count verified, ok[n])."""
    lf = np.ascontiguousarray(leaf, np.uint64)
    t = np.ascontiguousarray(terms, np.uint8)
    d = np.ascontiguousarray(digests, np.uint8)
    n, D = t.shape[0], t.shape[1]
    ok = np.zeros(max(n, 1), np.uint8)
    c = lib().orc_htree_verify_batch(n, _p(lf, u64p), width, _p(t), D, _p(d), _p(_u8(root)),
                                     _p(ok))
    return c, ok[:n]


def ahtree_verify_batch(kind, i, j, term_off, terms, a, b, nthreads=1):
    """kind 0/1/2 = VerifyInclusion / VerifyConsistency / VerifyLastInclusion
    over CSR proofs: term_off (n+1,) u64 in terms, terms (T,32), a/b (n,32).
    Returns (count verified, ok[n])."""
    iv = np.ascontiguousarray(i, np.uint64)
    jv = np.ascontiguousarray(j, np.uint64)
    to = np.ascontiguousarray(term_off, np.uint64)
    t = np.ascontiguousarray(terms, np.uint8).reshape(-1, 32)
    if t.shape[0] == 0:
        t = np.zeros((1, 32), np.uint8)
    av = np.ascontiguousarray(a, np.uint8)
    bv = np.ascontiguousarray(b, np.uint8)
    n = iv.shape[0]
    ok = np.zeros(max(n, 1), np.uint8)
    c = lib().orc_ahtree_verify_batch(kind, n, _p(iv, u64p), _p(jv, u64p), _p(to, u64p), _p(t),
                                      _p(av), _p(bv), _p(ok), nthreads)
    return c, ok[:n]


# ---------------------------------------------------------------- VerifyDocument
ERR_ILLEGAL_ARGS = 2
ERR_INVALID_PROOF = 20
ERR_UNSUPPORTED_TX_VERSION = 21
ERR_INVALID_PROOF_ENTRY = 22
_EMPTY = bytes.fromhex("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")


def verify_document(d, md_blob=b""):
    """pkg/verification.VerifyDocument (pkg/verification/verification.go:37-196),
    the hashing part, restated over the oracle's primitives.  d: the dict of
    immustore_amd.txlayer.verify_document_batch.  -> (status, target_alh or None).
    Not restated (the caller's, not hashing): the document-id lookup and
    encodedKeyForDocument (:50-58), the document decode + proto.Equal
    (:78-110), the signature check (:199-205)."""
    doc, key = bytes(d["encoded_document"]), bytes(d["doc_key"])
    # :60-76 -- the document's entry must exist exactly once with HValue = SHA256(doc)
    found = 0
    for ek, _, hv in d["entries"]:
        if bytes(ek) == key:
            if bytes(hv) != sha256(doc):
                return ERR_INVALID_PROOF_ENTRY, None
            found += 1
    if found != 1:
        return ERR_INVALID_PROOF_ENTRY, None
    tx = np.asarray(d["tx_hdr"], TX_HEADER).reshape(1)[0]
    ver = int(tx["version"])
    # :118-121 EntrySpecDigestFor (store/verification.go:244-254)
    if ver not in (0, 1):
        return ERR_UNSUPPORTED_TX_VERSION, None
    digs = []
    for ek, md, hv in d["entries"]:
        if ver == 0:
            # EntrySpecDigest_v0 (store/verification.go:256-262): key || SHA256(Value),
            # Value nil in VerifyDocument's EntrySpec -> SHA256(nil); md ignored
            digs.append(sha256(bytes(ek) + _EMPTY))
        else:
            # EntrySpecDigest_v1 (:264-302), IsValueTruncated -> HashValue
            st, dg = entry_digest(1, bytes(ek), bytes(md), bytes(hv))
            assert st == 0
            digs.append(dg)
    root = htree_build(np.frombuffer(b"".join(digs), np.uint8).reshape(-1, 32))[1] if digs \
        else _EMPTY
    if root != bytes(tx["eh"]):  # :137-139
        return ERR_INVALID_PROOF, None
    sh = np.asarray(d["src_hdr"], TX_HEADER).reshape(1).copy()
    th = np.asarray(d["tgt_hdr"], TX_HEADER).reshape(1).copy()
    x = np.asarray(d["tx_hdr"], TX_HEADER).reshape(1).copy()
    for h in (sh, th, x):  # a v0 innerHash never reads the metadata (tx.go:258-263)
        if int(h[0]["version"]) == 0:
            h[0]["md_len"] = 0
    src, tgt = int(sh[0]["id"]), int(th[0]["id"])
    if tgt < src:  # :146-148
        return ERR_INVALID_PROOF, None
    s1, _, salh = tx_header_alh(sh[0], md_blob)
    s2, _, talh = tx_header_alh(th[0], md_blob)
    if s1 or s2:  # Go's innerHash panics on such a header
        return ERR_ILLEGAL_ARGS, None
    tid = int(x[0]["id"])
    if tid != src and tid != tgt:  # :153-155
        return ERR_INVALID_PROOF, None
    s3, _, xalh = tx_header_alh(x[0], md_blob)
    if s3:
        return ERR_ILLEGAL_ARGS, None
    if (tid == src and xalh != salh) or (tid == tgt and xalh != talh):  # :157-163
        return ERR_INVALID_PROOF, None
    kid = int(d.get("known_tx_id", 0))
    ka = bytes(d.get("known_alh", bytes(32)))
    if kid == 0:
        if src != 1:  # :165-168
            return ERR_INVALID_PROOF, None
    else:
        if kid != src and kid != tgt:  # :170-172
            return ERR_INVALID_PROOF, None
        if (kid == src and ka != salh) or (kid == tgt and ka != talh):  # :174-180
            return ERR_INVALID_PROOF, None
    st = verify_dual_proof_v2(sh[0], th[0], md_blob, d["incl"], d["cons"], src, tgt, salh, talh)
    return st, (talh if st == 0 else None)
