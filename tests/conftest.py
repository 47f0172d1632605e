import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: large (Reddit-shape) inputs")


@pytest.fixture(scope="session")
def tiny_cases():
    """{case: {rows, cols, vals, n, X, Y0..Y3}} made by tests/golden/gen_golden.py
    from the reference's own sgc_precompute."""
    z = np.load(os.path.join(GOLDEN, "tiny_cases.npz"))
    cases = {}
    for key in z.files:
        name, field = key.split("/")
        cases.setdefault(name, {})[field] = z[key]
    return cases


@pytest.fixture(scope="session")
def shapes_golden():
    with open(os.path.join(GOLDEN, "shapes.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def shape_rows():
    return dict(np.load(os.path.join(GOLDEN, "shape_rows.npz")))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o
