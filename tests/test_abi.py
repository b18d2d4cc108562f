"""CPU-side checks of the drop-in boundary (no GPU needed).

- the C-ABI library builds for gfx950 and exports every symbol declared in
  include/immustore_merkle.h
- the ctypes mirror declares exactly that symbol set
- pure host-side index math (levels layout, nodesUpto) agrees with the oracle
- without a device the product fails loudly (no silent CPU fallback)
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "immustore_merkle.h")
LIB = os.path.join(ROOT, "immustore_amd", "libimmustore_merkle.so")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(mh_[a-z0-9_]+)\s*\(", src))


@pytest.fixture(scope="module")
def lib_built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "immustore_amd", "csrc"), "-j4"],
                       check=True)
    return LIB


def test_exports_match_header(lib_built):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_built], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (mh_[a-z0-9_]+)", out))
    declared = header_symbols()
    assert declared, "no declarations parsed"
    assert declared - exported == set(), "declared but not exported"
    assert exported - declared == set(), "exported but not declared"


def test_ctypes_mirror_matches_header(lib_built):
    from immustore_amd import _native
    assert set(_native.SIGNATURES) == header_symbols()
    L = _native.load()
    for name in _native.SIGNATURES:
        assert hasattr(L, name)


def test_gfx950_code_object(lib_built):
    blob = open(lib_built, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_host_index_math(lib_built, orc):
    import immustore_amd as m
    for n in list(range(0, 70)) + [1000, 1023, 1024, 1025, 4097, 1 << 20, (1 << 20) + 3]:
        assert m.levels_len(n) == orc.levels_len(n)
        for lvl in range(0, 22):
            if n and lvl < max(1, (n - 1).bit_length() + 1):
                assert m.level_offset(n, lvl) == orc.level_offset(n, lvl)
    for n in list(range(1, 200)) + [10 ** 7, 2 ** 40 + 12345]:
        assert m.nodes_upto(n) == orc.nodes_upto(n)
    # BASELINE C3: 10^7 appends -> 124,434,624 dLog digests
    assert m.nodes_upto(10 ** 7) == 124434624


def test_no_silent_cpu_fallback(lib_built):
    import torch  # noqa: F401  (same HIP runtime as the GPU box)
    import immustore_amd as m
    if m.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(m.ErrNoDevice):
        m.Context(0)
