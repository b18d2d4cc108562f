"""CSR batches of transactions for the precommit tests (host + GPU).

fixture_batch: the Go-written stores' transactions (tests/golden), with
optionally every k-th value replaced by its stored hVal as a truncated value
(EntrySpec.IsValueTruncated, immustore.go:1624-1626); the stored header Eh is
the expected result.  random_batch: seeded ragged batches (empty txs, long
and empty values, KV metadata, truncated values)."""
import numpy as np


def _csr(items):
    off = np.zeros(len(items) + 1, np.uint64)
    if items:
        off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    flat = b"".join(items)
    return (np.frombuffer(flat, np.uint8).copy() if flat else np.zeros(1, np.uint8)), off


def pack(txs):
    """txs: list of lists of (key, md, value, override-or-None) -> kwargs."""
    tx_off = np.zeros(len(txs) + 1, np.uint64)
    ents = []
    for t, es in enumerate(txs):
        ents.extend(es)
        tx_off[t + 1] = len(ents)
    keys, key_off = _csr([e[0] for e in ents])
    md, md_off = _csr([e[1] for e in ents])
    vals, val_off = _csr([e[2] for e in ents])
    out = dict(tx_off=tx_off, keys=keys, key_off=key_off, vals=vals, val_off=val_off)
    if any(len(e[1]) for e in ents):
        out.update(md=md, md_off=md_off)
    if any(e[3] is not None for e in ents):
        ov = np.zeros((max(len(ents), 1), 32), np.uint8)
        use = np.zeros(max(len(ents), 1), np.uint8)
        for k, e in enumerate(ents):
            if e[3] is not None:
                ov[k] = np.frombuffer(e[3], np.uint8)
                use[k] = 1
        out.update(hval_override=ov, use_override=use)
    return out


def fixture_batch(fx, truncate_every=0):
    txs, eh = [], []
    k = 0
    for tx in fx["txs"]:
        es = []
        for e in tx["entries"]:
            val = bytes.fromhex(e["value"])
            ov = None
            if truncate_every and k % truncate_every == 0:
                ov, val = bytes.fromhex(e["hval"]), b""
            es.append((bytes.fromhex(e["key"]), bytes.fromhex(e["md"]), val, ov))
            k += 1
        txs.append(es)
        eh.append(bytes.fromhex(tx["header"]["eh"]))
    version = fx["txs"][0]["header"]["version"]
    return version, pack(txs), np.frombuffer(b"".join(eh), np.uint8).reshape(-1, 32)


def random_batch(rng, ntx, version=1, max_entries=40, vlens=(0, 1, 55, 56, 64, 100, 1024, 3000),
                 md_prob=0.2, trunc_prob=0.1, empty_prob=0.05, klens=None):
    txs = []
    for _ in range(ntx):
        n = 0 if rng.random() < empty_prob else int(rng.integers(1, max_entries + 1))
        es = []
        for _ in range(n):
            kl = int(rng.choice(klens)) if klens is not None else int(rng.integers(1, 64))
            key = rng.integers(0, 256, kl, dtype=np.uint8).tobytes()
            md = b""
            if version == 1 and rng.random() < md_prob:
                md = rng.integers(0, 256, int(rng.integers(1, 12)), dtype=np.uint8).tobytes()
            val = rng.integers(0, 256, int(rng.choice(vlens)), dtype=np.uint8).tobytes()
            ov = None
            if rng.random() < trunc_prob:
                ov = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
            es.append((key, md, val, ov))
        txs.append(es)
    return pack(txs)
