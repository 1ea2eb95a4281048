"""Shared pytest configuration: the `gpu` marker and the golden fixtures."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_pattern(name: str) -> np.ndarray:
    """A shipped erasure pattern (one byte per packet, 1 = erased), e.g. 'bin_erasure'."""
    z = np.load(os.path.join(GOLDEN, "erasure_patterns.npz"))
    return np.unpackbits(z[name])[: int(z[name + "_len"][0])].astype(np.uint8)


def load_json(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def published_runs():
    return [r for r in load_json("published_fixed_logs.json")["runs"] if r["usable"]]


@pytest.fixture(scope="session")
def oracle_vectors():
    return load_json("oracle_vectors.json")
