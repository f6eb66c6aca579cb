import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


def _ensure_built():
    lib = os.path.join(ROOT, "bitflood_amd", "lib", "liblbfhash.so")
    orc = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "bitflood_amd", "csrc")])


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    def load(name):
        with open(os.path.join(GOLDEN, name)) as f:
            return json.load(f)
    return load


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def hasher():
    """A GPU context; GPU tests only."""
    from bitflood_amd import ChunkHasher
    h = ChunkHasher()
    yield h
    h.close()
