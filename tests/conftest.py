import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The suite runs the library's own (production) schedule; the non-production forms are
# explicit parametrisations (cases.py ALL_FORMS, apply_schedule).
for p in (os.path.join(REPO, "cs184-raytracer_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity of the HIP path vs the oracle")
    config.addinivalue_line("markers", "slow: long-running (large images)")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(REPO, "tests", "golden", "ref_hashes.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def rt():
    import rtamd
    rtamd.lib()
    return rtamd


@pytest.fixture(scope="session")
def gpu(rt):
    if rt.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X (no CPU fallback exists)")
    return rt
