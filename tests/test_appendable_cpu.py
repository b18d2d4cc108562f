"""The appendable framing of the ahtree logs (capi_app.hip, SURVEY.md 8(f)
row 4) against the reference's Go-written stores: the singleapp header of
aht/{data,tree,commit}/00000000.* (single_app.go:116-171, metadata.go:33-110,
multi_app.go:152-154, ahtree.go:106-107), kept as data in
tests/golden/immudb_fixtures.json, and the multiapp file addressing
(multi_app.go:204-214).  Host code of the C ABI: runs on the CPU."""
import struct

import numpy as np
import pytest


def parse_metadata(b: bytes) -> dict:
    """appendable.Metadata.ReadFrom (metadata.go:44-70): field(BE32 count),
    then field(key) field(value) per entry, field = BE32 len || bytes."""
    def field(p):
        n = struct.unpack(">I", b[p:p + 4])[0]
        return b[p + 4:p + 4 + n], p + 4 + n
    cnt, p = field(0)
    out = {}
    for _ in range(struct.unpack(">I", cnt)[0]):
        k, p = field(p)
        v, p = field(p)
        out[k.decode()] = v
    assert p == len(b)
    return out


def parse_header(h: bytes) -> dict:
    """singleapp header -> nested dict (WRAPPED_METADATA expanded)."""
    ml = struct.unpack(">I", h[:4])[0]
    assert len(h) == 4 + ml

    def expand(m):
        return {k: (expand(parse_metadata(v)) if k == "WRAPPED_METADATA" else v)
                for k, v in m.items()}
    return expand(parse_metadata(h[4:]))


@pytest.fixture(scope="module")
def app():
    from immustore_amd import appendable
    return appendable


def test_header_matches_go_written_files(app, fixtures):
    seen = 0
    for name, fx in fixtures.items():
        for rel, hx in fx["app_headers"].items():
            go = bytes.fromhex(hx)
            g = parse_header(go)
            fs = struct.unpack(">q", g["WRAPPED_METADATA"]["FILE_SIZE"])[0]
            cf = struct.unpack(">q", g["COMPRESSION_FORMAT"])[0]
            cl = struct.unpack(">q", g["COMPRESSION_LEVEL"])[0]
            pre = struct.unpack(">q", g["PREALLOC_SIZE"])[0] if "PREALLOC_SIZE" in g else -1
            ours = app.ahtree_log_header(fs, pre, cf, cl)
            # Go writes map order (differs file to file): same entries, same size
            assert parse_header(ours) == g, (name, rel)
            assert len(ours) == len(go), (name, rel)
            seen += 1
    assert seen == 9


def test_header_defaults_and_prealloc(app):
    h = parse_header(app.ahtree_log_header())
    assert h == {"COMPRESSION_FORMAT": bytes(8), "COMPRESSION_LEVEL": struct.pack(">q", 1),
                 "PREALLOC_SIZE": bytes(8),
                 "WRAPPED_METADATA": {"FILE_SIZE": struct.pack(">q", 1 << 26),
                                      "WRAPPED_METADATA": {"VERSION": struct.pack(">q", 1)}}}
    assert "PREALLOC_SIZE" not in parse_header(app.ahtree_log_header(1 << 20, -1))


def test_metadata_bytes_layout(app):
    assert app.metadata_bytes([]) == struct.pack(">II", 4, 0)
    b = app.metadata_bytes([("A", b"xy"), ("BC", b"")])
    assert b == struct.pack(">II", 4, 2) + struct.pack(">I", 1) + b"A" + struct.pack(">I", 2) + \
        b"xy" + struct.pack(">I", 2) + b"BC" + struct.pack(">I", 0)
    assert parse_metadata(b) == {"A": b"xy", "BC": b""}


def test_go_files_rebuilt_from_streams(app, fixtures):
    """Header + record stream = the Go-written file, entry order aside: the
    byte stream after the header is exactly the dLog / pLog / cLog."""
    for name, fx in fixtures.items():
        streams = {"aht/tree/00000000.sha": bytes.fromhex(fx["aht_dlog"]),
                   "aht/data/00000000.dat": bytes.fromhex(fx["aht_plog"]),
                   "aht/commit/00000000.di": bytes.fromhex(fx["aht_clog"])}
        for rel, data in streams.items():
            go = bytes.fromhex(fx["app_headers"][rel])
            g = parse_header(go)
            fs = struct.unpack(">q", g["WRAPPED_METADATA"]["FILE_SIZE"])[0]
            hdr = app.ahtree_log_header(fs, -1, 0, 1)
            files = {}
            app.write_range(files, 0, data, fs, hdr)
            assert list(files) == ([0] if data else [])
            if data:
                assert bytes(files[0][len(hdr):]) == data


@pytest.mark.parametrize("file_size", [1, 7, 32, 100, 4096])
def test_multiapp_segments_split_and_rebuild(app, file_size):
    """appendableID = off / fileSize and the in-file offset off % fileSize
    (multi_app.go:208-214) behind the header; appending ranges one after
    another rebuilds every file as the multiapp would write it."""
    rng = np.random.default_rng(file_size)
    log = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    hdr = app.ahtree_log_header(file_size)
    files = {}
    off = 0
    for n in (0, 1, 31, 32, 33, 700, 1, 4096 - 794, 200):
        if off + n > len(log):
            break
        app.write_range(files, off, log[off:off + n], file_size, hdr)
        off += n
    for fid, f in files.items():
        lo = fid * file_size
        assert bytes(f[:len(hdr)]) == hdr
        assert bytes(f[len(hdr):]) == log[lo:min(lo + file_size, off)], fid
    assert sorted(files) == list(range(-(-off // file_size)))
    segs = app.multiapp_segments(95, 210, 100, 10)
    assert segs == [(0, 105, 0, 5), (1, 10, 5, 100), (2, 10, 105, 100), (3, 10, 205, 5)]
    assert app.multiapp_segments(7, 0, 100, 10) == []
    assert app.file_name("tree", 3) == "tree/00000003.sha"
