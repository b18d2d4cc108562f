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
    assert len(calls) >= 18
    names = {n for _, n, _ in calls}
    # the store shim's PCIe-bound batches run over the process-wide clique
    assert {"mh_multi_create", "mh_multi_txlog_validate", "mh_multi_verify_values_batch",
            "mh_multi_precommit_batch", "mh_multi_ahtree_append_batch"} <= names
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


def _func_body(path, name):
    """Source of Go function `name` (from its `func` line to the closing brace
    at column 0)."""
    src = open(os.path.join(GO, path)).read()
    m = re.search(r"^func (\([^)]*\) )?%s\(" % re.escape(name), src, flags=re.M)
    assert m, "%s not in %s" % (name, path)
    end = src.index("\n}\n", m.start())
    return src[m.start():end + 2]


def test_verify_inclusion_batch_guards():
    """htree.VerifyInclusion returns false for a nil proof (htree.go:167-169):
    the batch shim skips nil proofs without touching C, and checks that
    digests / roots hold one entry per proof before C reads n x 32 bytes."""
    b = _func_body("htree/htree_mi355x.go", "VerifyInclusionBatch")
    assert re.search(r"len\(digests\) != n \|\| len\(roots\) != n", b)
    assert re.search(r"if pr != nil", b)
    # only the packed non-nil proofs reach the C call
    call = b[b.index("C.mh_htree_verify_inclusion_batch"):]
    assert "C.uint64_t(m)" in call and "&dig[0][0]" in call and "&rts[0][0]" in call
    assert b.index("if pr != nil") < b.index("mi355x.Context()")


def test_ahtree_append_batch_accepts_mixed_lengths():
    """Append accepts any non-nil payload (ahtree.go:260-263): AppendBatch
    rejects only nil, cuts runs of equal length, and passes no payload
    pointer for zero-length payloads."""
    b = _func_body("ahtree/ahtree_mi355x.go", "AppendBatch")
    assert "len(d) != plen" not in b
    assert re.search(r"if d == nil \{\s*return 0, root, ErrIllegalArguments", b)
    assert "t.appendRun(ds[i:j])" in b
    r = _func_body("ahtree/ahtree_mi355x.go", "appendRun")
    assert re.search(r"if plen > 0 \{\s*pp = ", r)
    assert "pp, C.uint64_t(m), C.uint32_t(plen)" in r


def test_verify_values_length_guards():
    b = _func_body("store/precommit_mi355x.go", "VerifyValues")
    assert re.search(r"len\(vLen\) != n \|\| len\(hVal\) != n", b)
    assert b.index("len(vLen) != n") < b.index("C.mh_multi_verify_values_batch")


def test_batch_paths_check_cliques_out_of_the_pool():
    """each batch call of the store / ahtree shims checks a
    clique out of the process's pool (mi355x.AcquireClique) and returns it
    (ReleaseClique, with the call's status so a clique whose collectives
    aborted is replaced) -- no process-wide shared handle is
    left, and no return between the checkout and the C call leaks it."""
    dev = open(os.path.join(GO, "internal/mi355x/device.go")).read()
    assert "func Multi(" not in dev
    acq = _func_body("internal/mi355x/device.go", "AcquireClique")
    assert "C.mh_multi_create" in acq and "poolCond.Wait()" in acq
    rel = _func_body("internal/mi355x/device.go", "ReleaseClique")
    assert "C.MH_ERR_COLLECTIVE" in rel and "C.mh_multi_destroy" in rel
    for path, fn, call in (("store/precommit_mi355x.go", "Run", "C.mh_multi_precommit_batch"),
                           ("store/precommit_mi355x.go", "VerifyValues",
                            "C.mh_multi_verify_values_batch"),
                           ("store/precommit_mi355x.go", "ValidateTxLog",
                            "C.mh_multi_txlog_validate"),
                           ("store/precommit_mi355x.go", "ValidateTxLogFromCommitLog",
                            "C.mh_txlog_validate_clog"),
                           ("ahtree/ahtree_mi355x.go", "appendRun",
                            "C.mh_multi_ahtree_append_batch")):
        b = _func_body(path, fn)
        a = b.index("AcquireClique()" if "AcquireClique()" in b else "devices()")
        c = b.index(call)
        r = b.index("ReleaseClique(", c)
        assert a < c < r, (path, fn)
        # every return between the checkout and the call releases the clique
        # first (or a deferred release covers it)
        between = b[b.index("\n\t}", a) + 3:c]  # after the checkout's own error return
        if "defer func()" not in between:
            for m_ in re.finditer(r"\n\s*return ", between):
                seg = between[:m_.start()]
                assert seg.rfind("ReleaseClique(") > seg.rfind("if err"), (path, fn)
    src = open(os.path.join(GO, "store/precommit_mi355x.go")).read()
    assert "mi355x.Multi" not in src and "b.multi" not in src
