import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rust-simd-r-drive_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        meta = json.load(f)
    out = {}
    for name, m in meta.items():
        with open(os.path.join(GOLDEN, m["file"]), "rb") as f:
            out[name] = (f.read(), m)
    return out


@pytest.fixture(scope="session")
def golden_cases():
    return load_cases()


@pytest.fixture(scope="session")
def ref_goldens():
    with open(os.path.join(GOLDEN, "reference_goldens.json")) as f:
        return json.load(f)
