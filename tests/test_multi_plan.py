"""The multi-GPU shard plan of the C ABI (mh_multi_shard_plan, host code, no
device) against sharding.shard_range, and the level assembly rule of
mh_multi_htree_build_entries_fixed checked with the oracle: the global
levels 0..log2 S restricted to shard g are the shard's own levels (its root
promoted above its own top, htree.go:100-103), the levels above are the tree
over the G shard roots -- for every (n, K) below, equal to the oracle's build
of the whole tree (finding 3)."""
import numpy as np
import pytest

from immustore_amd import multi, sharding


@pytest.mark.parametrize("K", [1, 2, 3, 4, 5, 8])
def test_shard_plan_matches_python_plan(K):
    for n in list(range(0, 70)) + [1023, 1024, 1025, 65535, 65536, 65537, (1 << 26) + 1]:
        S, G = multi.shard_plan(n, K)
        if n == 0:
            assert G == 0
            continue
        assert S & (S - 1) == 0 and S * K >= n and (S == 1 or (S // 2) * K < n)
        assert G == -(-n // S) and G <= K
        for r in range(K):
            lo, hi = sharding.shard_range(r, K, n)
            assert (lo, hi) == (min(r * S, n), min(r * S + S, n))


@pytest.mark.parametrize("K", [2, 3, 4, 8])
def test_level_assembly_rule_vs_oracle(orc, K):
    rng = np.random.default_rng(K)
    for n in (2, 3, 5, 9, 17, 100, 257, 1000, 4097):
        d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        glv, groot = orc.htree_build(d)
        S, G = multi.shard_plan(n, K)
        kS = S.bit_length() - 1
        out = np.zeros_like(glv)
        top = []
        for g in range(G):
            lo = g * S
            ng = min(S, n - lo)
            lv, r = orc.htree_build(d[lo:lo + ng])
            top.append(np.frombuffer(r, np.uint8))
            nl = max(ng - 1, 0).bit_length() + 1
            gnl = (n - 1).bit_length() + 1  # levels of the whole tree
            for l in range(0, min(kS, gnl - 1) + 1):
                ll = min(l, nl - 1)
                w = -(-ng // (1 << l)) if l < nl else 1
                src = lv[orc.level_offset(ng, ll):orc.level_offset(ng, ll) + w]
                dst = orc.level_offset(n, l) + (lo >> l)
                out[dst:dst + w] = src
        if G > 1:
            # the levels above: node hashes only over the G shard roots
            # (htree.go:85-110 without the leaf step; mh_dev_htree_reduce_nodes)
            cur = [bytes(t) for t in top]
            j = 0
            while len(cur) > 1:
                cur = [orc.sha256(b"\x01" + cur[i] + cur[i + 1]) if i + 1 < len(cur) else cur[i]
                       for i in range(0, len(cur), 2)]
                j += 1
                o = orc.level_offset(n, kS + j)
                out[o:o + len(cur)] = np.frombuffer(b"".join(cur), np.uint8).reshape(-1, 32)
            assert cur[0] == groot
        assert np.array_equal(out, glv), (n, K)
