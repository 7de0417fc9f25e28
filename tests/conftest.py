import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    """(manifest cases, npz arrays) restated from the reference's test suite."""
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "manifest.json")) as f:
        man = json.load(f)
    arrs = np.load(os.path.join(d, "golden.npz"), allow_pickle=False)
    return man["cases"], arrs
