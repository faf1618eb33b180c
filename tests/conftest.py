import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "token_vectors.json")
GOLDEN_HKDF = os.path.join(ROOT, "tests", "golden", "hkdf_vectors.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU and librnstok.so (run with -m gpu)")
    config.addinivalue_line("markers", "reference: needs the reference checkout at /root/reference (build container only)")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_hkdf():
    import json
    with open(GOLDEN_HKDF) as f:
        return json.load(f)
