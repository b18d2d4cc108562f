"""Argument checking of every C-ABI entry point ("nothing aborts across the
ABI", include/immustore_merkle.h): each int-returning function is called with
NULL handles / pointers and must return a status, never crash.

- CPU (no device): all-zero arguments -- NULL context / handles / pointers.
- GPU: a live context, NULL pointers and non-zero sizes (3), for every
  function whose first parameter is `mh_ctx *` (read from the header): the
  argument checks must reject the call before anything is launched or copied.
"""
import ctypes as C

import pytest

OK = {0, 2}  # MH_OK, MH_ERR_ILLEGAL_ARGUMENTS


def _zero_args(argtypes, fill_int=0, ctx=None):
    args = []
    for k, t in enumerate(argtypes):
        if k == 0 and ctx is not None:
            args.append(ctx)
        elif t in (C.c_void_p, C.c_char_p) or (isinstance(t, type) and issubclass(t, C._Pointer)):
            args.append(None)
        else:
            args.append(t(fill_int))
    return args


def test_null_arguments_without_device():
    from immustore_amd import _native as N
    L = N.load()
    for name, (res, argtypes) in N.SIGNATURES.items():
        if res is not C.c_int or name == "mh_abi_version":
            continue
        rc = getattr(L, name)(*_zero_args(argtypes))
        # a NULL handle is rejected first; the few calls that reach the HIP
        # runtime without a device report its error (negative) or no device
        assert rc in OK or rc == N.MH_ERR_NO_DEVICE or rc < 0, (name, rc)


# functions that must not get a live ctx with NULL buffers (they would
# destroy it, or hand NULL to the runtime's copy engine)
_SKIP_GPU = {"mh_abi_version", "mh_ctx_destroy", "mh_memcpy_h2d", "mh_memcpy_d2h", "mh_ctx_create",
             "mh_host_alloc_pinned", "mh_host_free_pinned", "mh_device_count", "mh_txlog_scan",
             "mh_dev_free"}


def _ctx_first_functions():
    """names of the entry points whose first parameter is `mh_ctx *` (header)."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "immustore_merkle.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\bint\s+(mh_[a-z0-9_]+)\s*\(\s*mh_ctx\s*\*", src))


@pytest.mark.gpu
def test_null_pointers_with_live_context():
    import torch  # noqa: F401
    import immustore_amd as m
    from immustore_amd import _native as N
    if m.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    L = N.load()
    ctx = m.Context(0)
    try:
        checked = 0
        ctx_first = _ctx_first_functions()
        for name, (res, argtypes) in N.SIGNATURES.items():
            if res is not C.c_int or name in _SKIP_GPU or name not in ctx_first:
                continue
            rc = getattr(L, name)(*_zero_args(argtypes, fill_int=3, ctx=ctx.handle))
            assert rc in OK, (name, rc)
            checked += 1
        ctx.synchronize()
        assert checked >= 30
    finally:
        ctx.close()


def _first_param_functions(kind):
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "immustore_merkle.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\bint\s+(mh_[a-z0-9_]+)\s*\(\s*" + kind + r"\s*\*", src))


@pytest.mark.gpu
def test_null_pointers_with_live_handles():
    """Entry points taking an mh_htree / mh_ahtree / mh_commit_pipe handle:
    live (empty) handles, NULL pointers, sizes 3 -> a Go sentinel status."""
    import torch  # noqa: F401
    import immustore_amd as m
    from immustore_amd import _native as N
    if m.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    L = N.load()
    ctx = m.Context(0)
    handles = {}
    try:
        for kind, mk in (("mh_htree", lambda h: L.mh_htree_new(ctx.handle, 1024, C.byref(h))),
                         ("mh_ahtree", lambda h: L.mh_ahtree_new(ctx.handle, C.byref(h))),
                         ("mh_commit_pipe",
                          lambda h: L.mh_commit_pipe_new(ctx.handle, 0, C.byref(h)))):
            h = C.c_void_p()
            N.check(mk(h))
            handles[kind] = h
        allowed = {0, 2, 3, 4, 5, 7, 19}
        checked = 0
        for kind, h in handles.items():
            for name in sorted(_first_param_functions(kind)):
                if name.endswith("_free"):
                    continue
                res, argtypes = N.SIGNATURES[name]
                rc = getattr(L, name)(*_zero_args(argtypes, fill_int=3, ctx=h))
                assert rc in allowed, (name, rc)
                checked += 1
        assert checked >= 20
        ctx.synchronize()
    finally:
        L.mh_htree_free(handles.get("mh_htree"))
        L.mh_ahtree_free(handles.get("mh_ahtree"))
        L.mh_commit_pipe_free(handles.get("mh_commit_pipe"))
        ctx.close()
