import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(TESTS, "golden")
ORACLE = os.path.join(ROOT, "oracle")  # test infrastructure (xdrc_front.py)
for p in (ROOT, TESTS, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libxdrgpu.so)")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLD, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLD, "kat.json")) as f:
        return json.load(f)


def golden(schema: str, n: int, ext: str, dtype=np.uint8) -> np.ndarray:
    return np.fromfile(os.path.join(GOLD, f"{schema}_{n}.{ext}"), dtype=dtype)


SMALL_N = {"numerics": 1000, "rec128": 1024, "recvar": 1024, "rpc": 1024, "vecrec": 1024,
           "containertest": 1024, "rp_list": 1024}


@pytest.fixture(scope="session")
def dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
