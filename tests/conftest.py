"""Shared test setup. `-m gpu` tests need a gfx950 device and the built HIP library; the
CPU suite (`-m "not gpu"`) covers the oracle against golden vectors, the host setup math and the
C-ABI library's exports."""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "sphereflake-raytracer_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")


def load_frame(name):
    with open(os.path.join(GOLDEN, f"frame_{name}.json")) as f:
        return json.load(f)


def load_progressive(name):
    with open(os.path.join(GOLDEN, f"progressive_{name}.json")) as f:
        return json.load(f)


def load_npz(name):
    return dict(np.load(os.path.join(GOLDEN, f"frame_{name}.npz")))


@pytest.fixture(scope="session")
def lut():
    return np.fromfile(os.path.join(GOLDEN, "rsqrtps_lut.bin"), dtype="<u4")
