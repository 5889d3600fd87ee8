"""Test configuration.

Markers:
  gpu  -- needs an MI355X (runs on the GPU box: `pytest -m gpu`).
Everything else runs on the CPU in this container (`pytest -m "not gpu"`).
The CPU checker (oracle/) is test infrastructure: tests import it only as the
thing results are compared against.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD MI355X GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def load_golden(name):
    path = os.path.join(GOLDEN, name)
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def golden_summary():
    import json
    with open(os.path.join(GOLDEN, "summary.json")) as f:
        return json.load(f)
