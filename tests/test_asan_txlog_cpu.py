"""Mutation fuzzing of the tx-log record hop under AddressSanitizer (CPU).

The hop (mh_txlog_scan, the host parse in front of mh_txlog_validate) reads
tx-log bytes from disk or a replica, tx.go:419-603, so it must stop with the
reader's error on any input and never read outside the buffer.
tools/asan/txlog_fuzz.c mutates the reference's Go-written tx logs, the
synthetic and metadata logs of tests/tx_util.py and a > 8 MiB log that takes
the multi-threaded hop (bit flips, extreme BE16 / BE32 length fields,
truncation, splices).  Each mutant sits in an allocation of its exact length;
the library's host code and the oracle are both built with ASan (host only,
tools/asan/Makefile), and the two parses must agree on (status, ntx,
consumed) for every mutant.  (tools/gpu_run.sh fuzz runs the same fuzzer on a GPU
box with the device path, mh_txlog_validate, compared in full:
profiles/fuzz_txlog_device_r02.log.)"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FUZZ = os.path.join(ROOT, "build", "asan", "txlog_fuzz")


def test_txlog_hop_fuzz_asan(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("host-sanitizer run: CPU container only")
    if not shutil.which("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "tools", "asan")], check=True,
                   timeout=600)
    sys.path.insert(0, os.path.join(ROOT, "tools", "asan"))
    import make_corpus
    make_corpus.main(str(tmp_path))
    files = sorted(str(p) for p in tmp_path.glob("*.log"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=86")
    r = subprocess.run([FUZZ, "1500", "20261016"] + files, capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == len(files)
    for line in lines:
        _, _, rest = line.partition(": ")
        n, agree = int(rest.split()[0]), int(rest.split(", ")[1].split()[0])
        assert n == agree and n > 0, line
