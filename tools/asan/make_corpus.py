"""Seed logs for tools/asan/txlog_fuzz: the reference's Go-written tx logs
(tests/golden/immudb_fixtures.json), the synthetic and metadata logs of
tests/tx_util.py and a > 8 MiB log that takes the multi-threaded hop.
usage: python tools/asan/make_corpus.py <out dir>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]

import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
from tx_util import _bulk_txlog, _synthetic_txlog, metadata_logs  # noqa: E402


def main(out):
    os.makedirs(out, exist_ok=True)
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "immudb_fixtures.json")))
    logs = {"fx_%s.log" % k: bytes.fromhex(v["txlog"]) for k, v in fx.items()}
    logs["synthetic.log"] = _synthetic_txlog(np.random.default_rng(5), 60, orc)
    for name, raw in metadata_logs(orc):
        logs["md_%s.log" % name] = raw
    logs["bulk.log"] = _bulk_txlog(np.random.default_rng(78), 9000)[0]
    for name, raw in logs.items():
        with open(os.path.join(out, name), "wb") as f:
            f.write(raw)
    print(len(logs), "logs in", out)


if __name__ == "__main__":
    main(sys.argv[1])
