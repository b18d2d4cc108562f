"""Every name a function of the bench / package / oracle / tool scripts reads
is bound somewhere: a local, an enclosing function's local, a module global
or a builtin (`bench_workloads.py --workload c5` under
torch.distributed read a `leaf_t` bound only in another function and raised
NameError on its first step -- a path no CPU test executes, since it needs a
GPU).  symtable classifies every name of every scope at compile time, so this
catches such a name on every path without running it (the pyflakes check,
with the standard library only)."""
import builtins
import glob
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(
    [os.path.join(ROOT, f) for f in ("bench.py", "bench_workloads.py", "__graft_entry__.py")] +
    glob.glob(os.path.join(ROOT, "immustore_amd", "*.py")) +
    glob.glob(os.path.join(ROOT, "oracle", "*.py")) +
    glob.glob(os.path.join(ROOT, "tools", "*.py")) +
    glob.glob(os.path.join(ROOT, "tests", "*.py")) +
    glob.glob(os.path.join(ROOT, "tests", "golden", "*.py")))


def unbound_names(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module = {s.get_name() for s in top.get_symbols()
              if s.is_assigned() or s.is_imported() or s.is_namespace() or s.is_global()}
    known = module | set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__builtins__",
                                           "__spec__", "__loader__", "__package__"}
    bad = []

    def walk(t):
        if t.get_type() == "function":
            for s in t.get_symbols():
                if s.is_referenced() and s.is_global() and s.get_name() not in known:
                    bad.append("%s: %s() reads unbound %r" % (os.path.basename(path), t.get_name(),
                                                              s.get_name()))
        for c in t.get_children():
            walk(c)

    walk(top)
    return bad


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.relpath(p, ROOT))
def test_no_unbound_names(path):
    assert unbound_names(path) == []


def test_checker_catches_the_r04_bug(tmp_path):
    """The shape of the round-4 bug: a nested step() reading a name that the
    enclosing function never binds."""
    f = tmp_path / "x.py"
    f.write_text("def main():\n    ok = 1\n\n    def step():\n        return leaf_t, ok\n"
                 "    return step\n\n\ndef other():\n    leaf_t = 2\n    return leaf_t\n")
    assert unbound_names(str(f)) == ["x.py: step() reads unbound 'leaf_t'"]
