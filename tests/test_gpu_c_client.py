"""The C ABI driven from plain C (tests/c_client/mh_client.c, built by
__graft_entry__.build()): what a cgo shim does, with no Python or torch in the
process.  Its printed roots and proofs must equal the oracle's
(htree.go:64-164, ahtree.go:149-651) on the same deterministic inputs."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
CLIENT = os.path.join(HERE, "c_client", "mh_client")


def _inputs(w, m):
    d = ((np.arange(w * 32, dtype=np.uint64) * 131 + 7) & 0xFF).astype(np.uint8).reshape(w, 32)
    p = ((np.arange(m * 32, dtype=np.uint64) * 29 + 3) & 0xFF).astype(np.uint8).reshape(m, 32)
    return d, p


def _run(w, m):
    if not os.path.exists(CLIENT):
        pytest.fail("tests/c_client/mh_client not built (run __graft_entry__.build())")
    r = subprocess.run([CLIENT, str(w), str(m)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    out = {}
    for line in r.stdout.splitlines():
        k, _, v = line.partition(" ")
        out[k] = v
    assert "done" in out
    return out


def _entries(ne):
    """The ragged CSR batch mh_client.c builds (see the comment there)."""
    e = np.arange(ne, dtype=np.int64)

    def csr(lens, a, b, c):
        # byte j of entry e = (a e + b j + c) & 0xff
        off = np.zeros(ne + 1, np.uint64)
        off[1:] = np.cumsum(lens)
        ent = np.repeat(e, lens)
        j = np.arange(int(off[-1]), dtype=np.int64) - np.repeat(off[:-1].astype(np.int64), lens)
        return np.append(((a * ent + b * j + c) & 0xFF).astype(np.uint8), np.uint8(0)), off

    ms = [[b"", b"\x00", b"\x02", b"\x01" + int(x).to_bytes(8, "big")][x % 4] for x in range(ne)]
    mo = np.zeros(ne + 1, np.uint64)
    mo[1:] = np.cumsum([len(x) for x in ms])
    md = (np.frombuffer(b"".join(ms) + b"\0", np.uint8), mo)
    return csr(1 + (7 * e) % 40, 13, 5, 1), md, csr((37 * e) % 700, 3, 11, 0), *_ovr(ne)


def _ovr(ne):
    ov = ((np.arange(ne)[:, None] + np.arange(32)[None, :]) & 0xFF).astype(np.uint8)
    use = (np.arange(ne) % 5 == 0).astype(np.uint8)
    return ov, use


def _check_entries(out, ne):
    (kb, ko), (mb, mo), (vb, vo), ov, use = _entries(ne)
    st, hv, _, root = O.build_entries_csr(1, kb, ko, mb, mo, vb, vo, False, ov, use)
    assert st == 0
    assert out["entries_v1_root"] == root.hex()
    assert out["entries_v1_hval_mid"] == hv[ne // 2].tobytes().hex()
    assert out["entries_v1_hval_last"] == hv[ne - 1].tobytes().hex()
    st, _, _, root0 = O.build_entries_csr(0, kb, ko, None, None, vb, vo, False)
    assert st == 0 and out["entries_v0_root"] == root0.hex()
    assert out["entries_v0_md_rejected"] == "1"
    if ne >= 2:
        assert out["entries_backwards_rejected"] == "1"


def test_c_client_entries_inputs_pin_oracle():
    """CPU: the oracle side of the C-client entries check is self-consistent
    (the overridden entries' hVals are the override bytes)."""
    (kb, ko), (mb, mo), (vb, vo), ov, use = _entries(64)
    st, hv, _, _ = O.build_entries_csr(1, kb, ko, mb, mo, vb, vo, False, ov, use)
    assert st == 0
    assert (hv[use == 1] == ov[use == 1]).all()
    assert int(mo[-1]) == 16 * 0 + 16 * 1 + 16 * 1 + 16 * 9


@pytest.mark.gpu
@pytest.mark.parametrize("w,m", [(1000, 777), (1, 3), (2, 4), (4096, 1 << 13), (65537, 100003),
                                 (300, 1000)])
def test_c_client_matches_oracle(w, m):
    out = _run(w, m)
    d, p = _inputs(w, m)
    lv, root = O.htree_build(d)
    assert out["htree_root"] == root.hex()
    assert out["max_width_exceeded"] == "1"
    st, terms = O.htree_inclusion_proof(lv, w, w // 3)
    assert st == 0
    assert out["htree_proof"] == terms.tobytes().hex()
    assert out["htree_verify"] == "1"
    assert out["htree_verify_tampered"] == ("0" if len(terms) else "1")
    # server-side DualProofV2 messages over a self-linked store, verified from the
    # wire by the client call: all pass; a flipped last byte fails that proof only
    assert out["wire_verify_ok"] == "40/40"
    code, rest = out["wire_verify_tampered"].split()
    assert int(code) != 0 and rest == "39"
    assert out["multi3_wire_verify_equal"] == "1"  # the mh_multi_* split, from plain C

    t = O.AHtree(cap=m)
    t.append_batch(p)
    assert out["ahtree_size"] == str(m)
    assert out["ahtree_root"] == t.root_at(m)[1].hex()
    assert out["ahtree_root_half"] == t.root_at(m // 2)[1].hex()
    st, inc = t.inclusion_proof(m // 3, m)
    assert st == 0 and out["ahtree_incl"] == inc.tobytes().hex()
    st, cons = t.consistency_proof(m // 2, m)
    assert st == 0 and out["ahtree_cons"] == cons.tobytes().hex()
    assert out["empty_root_at"] == "1"
    for k in ("multi1_ahtree_root_equal", "multi1_ahtree_dlog_equal", "multi3_ahtree_root_equal",
              "multi3_ahtree_dlog_equal"):
        assert out[k] == "1", k
    _check_entries(out, w)
    if m >= 2 * w:
        # mh_multi_htree_build_entries_fixed (RCCL clique of device 0; three shards)
        keys = np.frombuffer(np.arange(w, dtype=">u8").tobytes(), np.uint8).reshape(w, 8)
        _, _, eroot = O.build_entries_fixed(1, keys, p[:2 * w].reshape(w, 64))
        assert out["multi1_root"] == eroot.hex() and out["multi3_root"] == eroot.hex()


def test_c_client_links_and_reports_no_device():
    """CPU: the C client resolves every ABI symbol it uses from the shared
    library and, without a device, fails through the ABI's status path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is visible: covered by the gpu test")
    subprocess.run(["make", "-s", "-C", os.path.dirname(CLIENT)], check=True)
    r = subprocess.run([CLIENT, "8", "8"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "abi 1" in r.stdout, (r.stdout, r.stderr)
    assert "mh_ctx_create" in r.stderr


COMMITTERS = os.path.join(HERE, "c_client", "mh_committers")


def _committer_batch(t, ntx, ne, vlen):
    """Thread t's batch in tests/c_client/mh_committers.c (see its comment)."""
    n = ntx * ne
    e = np.arange(n, dtype=np.int64)
    keys = np.frombuffer(((np.int64(t) << 32) | e).astype(">u8").tobytes(), np.uint8).copy()
    j = np.arange(vlen, dtype=np.int64)
    vals = ((7 * t + 13 * e[:, None] + 11 * j[None, :] + 1) & 0xFF).astype(np.uint8).reshape(-1)
    return dict(tx_off=np.arange(0, n + 1, ne, dtype=np.uint64), keys=keys,
                key_off=np.arange(0, 8 * n + 1, 8, dtype=np.uint64), vals=vals,
                val_off=np.arange(0, vlen * n + 1, vlen, dtype=np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("threads,cliques", [(4, 4), (4, 2), (3, 1)])
def test_concurrent_committers_clique_pool(threads, cliques):
    """Concurrent committers from plain C (one handle per
    concurrent committer): `threads` threads share a pool of `cliques`
    mh_multi handles over device 0 (checkout / return, as the cgo shim's
    AcquireClique / ReleaseClique) and run mh_multi_precommit_batch at once;
    every thread's Eh and sampled hVals equal the oracle's precommit
    (immustore.go:1620-1632)."""
    if not os.path.exists(COMMITTERS):
        pytest.fail("tests/c_client/mh_committers not built (run __graft_entry__.build())")
    ntx, ne, vlen, rounds = 48, 8, 300, 3
    r = subprocess.run([COMMITTERS, str(threads), str(cliques), str(rounds), str(ntx), str(ne),
                        str(vlen)], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    eh, hv = {}, {}
    for line in r.stdout.splitlines():
        k, *rest = line.split()
        if k == "eh":
            eh[int(rest[0])] = rest[1]
        elif k == "hv":
            hv[int(rest[0])] = rest[1]
    assert sorted(eh) == list(range(threads))
    n = ntx * ne
    for t in range(threads):
        h_o, e_o, st_o = O.precommit_batch(1, **_committer_batch(t, ntx, ne, vlen))
        assert not st_o.any()
        assert eh[t] == e_o.tobytes().hex(), t
        assert hv[t] == (h_o[0].tobytes() + h_o[n // 2].tobytes() + h_o[n - 1].tobytes()).hex(), t
