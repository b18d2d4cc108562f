"""The cgo shim (go/**/*.go) against the C ABI it binds:
every C.mh_* function and C.MH_* constant the Go files use is declared in
include/immustore_merkle.h, every call passes the header's number of
arguments, and every such function is exported by the built library.  The Go
files cannot be compiled here (no Go toolchain in the image); this is the
check that they bind the ABI as declared."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "immustore_merkle.h")
GO = os.path.join(ROOT, "go")


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def header_prototypes():
    """name -> parameter count of every function the header declares."""
    s = _strip_c_comments(open(HDR).read())
    out = {}
    for m in re.finditer(r"\b(mh_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", s, flags=re.S):
        name, params = m.group(1), m.group(2).strip()
        if not params or params == "void":
            out[name] = 0
        else:
            out[name] = params.count(",") + 1
    return out


def header_constants():
    s = open(HDR).read()
    return set(re.findall(r"#define\s+(MH_[A-Z0-9_]+)", s))


def _go_sources():
    files = []
    for d, _, fs in os.walk(GO):
        files += [os.path.join(d, f) for f in fs if f.endswith(".go")]
    return sorted(files)


def _split_args(s):
    """Top-level comma count of a Go argument list (parens / brackets /
    braces / string literals respected)."""
    depth, n, i, seen = 0, 0, 0, False
    while i < len(s):
        c = s[i]
        if c in "\"'`":
            j = i + 1
            while j < len(s) and s[j] != c:
                j += 2 if s[j] == "\\" and c != "`" else 1
            i = j + 1
            seen = True
            continue
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
        elif c == "," and depth == 0:
            n += 1
        if not c.isspace():
            seen = True
        i += 1
    return 0 if not seen else n + 1


def go_calls():
    """(file, name, argc) of every C.mh_*( call in the Go sources."""
    calls = []
    for f in _go_sources():
        src = open(f).read()
        body = src.split('import "C"', 1)[1] if 'import "C"' in src else src
        body = re.sub(r"//[^\n]*", "", body)
        for m in re.finditer(r"\bC\.(mh_[a-z0-9_]+)\s*\(", body):
            i, depth = m.end(), 1
            while depth and i < len(body):
                depth += {"(": 1, ")": -1}.get(body[i], 0)
                i += 1
            calls.append((os.path.relpath(f, ROOT), m.group(1), _split_args(body[m.end():i - 1])))
    return calls


def test_go_files_exist():
    names = {os.path.relpath(f, GO) for f in _go_sources()}
    for want in ("htree/htree_mi355x.go", "store/precommit_mi355x.go", "ahtree/ahtree_mi355x.go",
                 "internal/mi355x/device.go"):
        assert want in names
    for f in _go_sources():
        src = open(f).read()
        assert src.startswith("//go:build mi355x"), f
        assert 'import "C"' in src and '#include "immustore_merkle.h"' in src, f


def test_every_c_call_is_declared_with_its_arity():
    protos = header_prototypes()
    calls = go_calls()
    assert len(calls) >= 20
    for f, name, argc in calls:
        assert name in protos, "%s calls C.%s, not in the header" % (f, name)
        assert argc == protos[name], "%s: C.%s with %d args, header has %d" % (
            f, name, argc, protos[name])


def test_every_constant_is_declared():
    consts = header_constants()
    used = set()
    for f in _go_sources():
        used |= set(re.findall(r"\bC\.(MH_[A-Z0-9_]+)", open(f).read()))
    assert used, "the shim maps no status codes"
    assert used <= consts, sorted(used - consts)


def test_bound_functions_are_exported():
    lib = os.path.join(ROOT, "immustore_amd", "libimmustore_merkle.so")
    if not os.path.exists(lib):
        pytest.skip("library not built")
    L = ctypes.CDLL(lib)
    for _, name, _ in go_calls():
        assert hasattr(L, name), name
