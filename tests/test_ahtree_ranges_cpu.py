"""The ranged multi-device ahtree append (mh_multi_(dev_)ahtree_append_batch,
mh_dev_ahtree_append_range) on the CPU: the library's range plan
(mh_ahtree_range_plan, host code) and a pure-Python model of the four phases
the devices run, in which every device may only touch its own dLog range and
its 64-slot frontier -- checked against the oracle's single AppendBatch
(ahtree.go:246-373) for appends onto non-empty trees (the replay of
syncBinaryLinking, immustore.go:1198-1232, resumes at aht.Size()+1).  The
model asserts the decomposition's claims: a range reads nothing outside itself
but the peaks of its left end, range d > 0 needs no frontier before the piece
tree, and the ranges tile the new dLog stream."""
import hashlib

import numpy as np
import pytest

from immustore_amd import _native as N
from immustore_amd.multi import ahtree_range_plan, peaks_of


def _leaf(p):
    return hashlib.sha256(b"\x00" + bytes(p)).digest()


def _node(a, b):
    return hashlib.sha256(b"\x01" + a + b).digest()


def _tz(x):
    return (x & -x).bit_length() - 1


def model_append(n0, peaks, pay, K):
    """New dLog digests of appending the rows of pay onto a tree of n0 with
    the given peaks, computed range by range as the devices do."""
    L = N.load()
    up = L.mh_ahtree_nodes_upto
    idx = L.mh_ahtree_node_index
    total = len(pay)
    k, b = ahtree_range_plan(n0, total, K)
    G = len(b) - 1
    S = 1 << k
    old = {}
    q = 0
    for l in range(64):
        if (n0 >> l) & 1:
            old[l] = peaks[32 * q:32 * q + 32]
            q += 1
    dev = [dict() for _ in range(G)]
    fr = [dict(old) if d == 0 else {} for d in range(G)]

    def put(d, kk, l, h):
        i = idx(kk, l)
        assert up(b[d]) <= i < up(b[d + 1]), (d, kk, l)
        dev[d][i] = h

    def read(d, kk, l):
        if kk <= b[d]:
            assert l in fr[d], ("read outside the range, not a peak", d, kk, l)
            return fr[d][l]
        i = idx(kk, l)
        assert up(b[d]) <= i < up(b[d + 1]), (d, kk, l)
        return dev[d][i]

    # 1. leaves + perfect levels 1..k (all levels for one range)
    for d in range(G):
        lo, hi = b[d], b[d + 1]
        for n in range(lo + 1, hi + 1):
            put(d, n, 0, _leaf(pay[n - n0 - 1]))
        for l in range(1, (64 if G == 1 else k + 1)):
            e = ((lo >> l) + 1) << l
            while e <= hi:
                put(d, e, l, _node(read(d, e - (1 << (l - 1)), l - 1), read(d, e, l - 1)))
                e += 1 << l
    if G > 1:
        # 2. piece roots (level k) of every device, gathered
        pe0 = [x >> k for x in b]
        roots = {}
        for d in range(G):
            for E in range(pe0[d] + 1, pe0[d + 1] + 1):
                roots[E] = dev[d][idx(E * S, k)]
        # 3. the piece tree (old peaks at the slot N0 >> l' of each level)
        N0, Pend = n0 >> k, b[G] >> k
        lev = [{}]
        if (n0 >> k) & 1:
            lev[0][N0] = old[k]
        lev[0].update(roots)
        lp = 1
        while (Pend >> lp) and k + lp < 64:
            cur = {}
            j0 = N0 >> lp
            if (n0 >> (k + lp)) & 1:
                cur[j0] = old[k + lp]
            for j in range(j0 + 1, (Pend >> lp) + 1):
                cur[j] = _node(lev[lp - 1][2 * j - 1], lev[lp - 1][2 * j])
            lev.append(cur)
            lp += 1
        for d in range(G):
            for lp in range(1, len(lev)):
                for j, h in lev[lp].items():
                    e = j << (k + lp)
                    if b[d] < e <= b[d + 1] and e > n0:
                        put(d, e, k + lp, h)
            if d:
                for l in range(k, 64):
                    if (b[d] >> l) & 1:
                        fr[d][l] = lev[l - k][(b[d] >> k) >> (l - k)]
    # 4. spines
    for d in range(G):
        for n in range(b[d] + 1, b[d + 1] + 1):
            t = _tz(n)
            h = read(d, n, t)
            rest = ((n - 1) >> (t + 1)) << (t + 1)
            while rest:
                l = _tz(rest)
                h = _node(read(d, rest, l), h)
                t += 1
                put(d, n, t, h)
                rest &= rest - 1
    out = []
    for d in range(G):
        for i in range(up(b[d]), up(b[d + 1])):
            out.append(dev[d][i])
    assert len(out) == up(n0 + total) - up(n0)
    return b"".join(out)


@pytest.mark.parametrize("K", [1, 2, 3, 5, 8])
def test_ranged_model_vs_oracle(orc, K):
    rng = np.random.default_rng(K)
    N_all = 3000
    pay = orc.fill_random(32 * N_all, 11).reshape(N_all, 32)
    o = orc.AHtree(N_all)
    o.append_batch(pay)
    ref = np.frombuffer(o.dlog_bytes(), np.uint8).reshape(-1, 32)
    L = N.load()
    cases = [(0, 1), (0, 7), (0, 64), (0, 1000), (1, 1), (1, 999), (127, 1), (127, 130),
             (255, 700), (1023, 1977), (1000, 3), (1000, 2000)]
    cases += [(int(a), int(b)) for a, b in zip(rng.integers(0, 1500, 6), rng.integers(1, 1500, 6))]
    for n0, total in cases:
        pk = peaks_of(ref, n0)
        got = model_append(n0, pk, pay[n0:n0 + total], K)
        want = ref[L.mh_ahtree_nodes_upto(n0):L.mh_ahtree_nodes_upto(n0 + total)].tobytes()
        assert got == want, (K, n0, total)


def test_range_plan_properties():
    L = N.load()
    for n0 in (0, 1, 2 ** 13 - 1, 10 ** 6 + 3, 2 ** 40 + 12345):
        for total in (1, 2, 7, 100, 4097, 10 ** 7, 2 ** 26):
            for K in (1, 2, 3, 4, 7, 8, 16, 64):
                k, b = ahtree_range_plan(n0, total, K)
                G = len(b) - 1
                assert 1 <= G <= K
                assert b[0] == n0 and b[-1] == n0 + total
                assert all(x < y for x, y in zip(b, b[1:]))
                assert all(x % (1 << k) == 0 for x in b[1:-1])
                # S <= total / 8K: within 1/8 of an even split once ranges are big
                assert (8 << k) * K <= max(total, 8 * K) or k == 0
                if total >= 64 * K:
                    sizes = [y - x for x, y in zip(b, b[1:])]
                    assert G == K
                    even = total / K
                    assert max(sizes) <= even * 1.13 + 1, (n0, total, K, sizes)
    st = L.mh_ahtree_range_plan(0, 5, 65, None, None, None)
    assert st != 0
