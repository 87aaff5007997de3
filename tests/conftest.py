import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP C-ABI library)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def golden_names(prefix):
    return sorted(n[:-4] for n in os.listdir(GOLDEN) if n.startswith(prefix) and n.endswith(".npz"))


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (den if den > 0 else 1.0))


@pytest.fixture
def golden():
    return load_golden
