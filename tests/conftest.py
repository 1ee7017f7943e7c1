import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The GPU tests render small images: with the production threshold every shading launch there
# would trace light-major (api.cpp light_major_below), and the all-lights and fused-Phong
# forms the full-size renders use would go untested.  The suite defaults to no threshold;
# tests that exercise it set it explicitly (test_gpu_fuzz odd seeds, knob tests, the bench
# batch test).
os.environ.setdefault("RTAMD_LIGHT_MAJOR_BELOW", "0")
# likewise the one-stream issue of small replayed chunks (api.cpp one_stream_pixels): off by
# default so the multi-stream schedule stays covered; odd fuzz seeds and a knob test run it
os.environ.setdefault("RTAMD_ONE_STREAM_PIXELS", "0")
os.environ.setdefault("RTAMD_ONE_STREAM_LEVEL1", "0")  # and of plans of one traced level
# and a scene's first call on its own streams (api.cpp Lane::minimal borrows the scene's stream
# and shades in the chain's order): most tests render a scene once; the production-schedule
# tests, odd fuzz seeds and a knob test run the minimal first call
os.environ.setdefault("RTAMD_FIRST_CALL_MINIMAL", "0")
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
