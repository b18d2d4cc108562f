import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def fixtures():
    with open(os.path.join(GOLDEN, "immudb_fixtures.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def synthetic():
    with open(os.path.join(GOLDEN, "synthetic.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.lib()
    return oracle
