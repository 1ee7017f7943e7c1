"""The same-algorithm CPU baseline (oracle/cpu_bvh.cpp, bench.py cpu_baseline.same_algorithm).

It runs the HIP path's algorithm (LBVH, world-box culling, any-hit shadows, zero-term
decisions) on the host, so its rate is a fair CPU comparison.  It is a
baseline only if it computes the reference's image: every shipped scene must match the
oracle bit for bit, with the reference's ray counts.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from cases import REPO, SCENES, scene_files

CLI = os.path.join(REPO, "oracle", "cpu_bvh_cli")


@pytest.fixture(scope="module")
def cpu_bvh():
    import fcntl
    # one make at a time (pytest-xdist workers would otherwise race on the same binary)
    with open(os.path.join(REPO, "oracle", ".make.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "cpu_bvh_cli"], check=True)
    return CLI


def run(cli, scene, w, h, bdepth, tmp_path, rows=None):
    r0, r1, step = rows or (0, h, 1)
    out = tmp_path / "img.raw"
    p = subprocess.run([cli, scene, str(w), str(h), str(bdepth), "4", str(r0), str(r1), str(step), str(out)],
                       capture_output=True, text=True, check=True)
    n = len(range(r0, r1, step))
    return np.fromfile(out, dtype=np.float64).reshape(n, w, 3), json.loads(p.stdout)


@pytest.mark.parametrize("rel", scene_files())
def test_matches_oracle(oracle, cpu_bvh, tmp_path, rel):
    scene = os.path.join(SCENES, rel)
    w, h, bdepth = 40, 30, 6
    try:
        want, cnt = oracle.render(scene, w, h, bdepth=bdepth)
    except oracle.OracleError:
        pytest.skip("the reference rejects this scene")
    got, st = run(cpu_bvh, scene, w, h, bdepth, tmp_path)
    diff = int((got.view(np.uint64) != want.view(np.uint64)).any(axis=2).sum())
    assert diff == 0, f"{diff} pixels differ from the oracle"
    assert (st["trace_rays"], st["shadow_rays"]) == (cnt["trace_rays"], cnt["shadow_rays"])


def test_row_sample(oracle, cpu_bvh, tmp_path):
    """bench.py times an evenly spaced row sample: rows (r0, r1, step) in order."""
    scene = os.path.join(SCENES, "excess_inputs", "bunny.rti")
    rows = (3, 54, 5)
    want, cnt = oracle.render(scene, 96, 54, bdepth=4, rows=rows)
    got, st = run(cpu_bvh, scene, 96, 54, 4, tmp_path, rows=rows)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    assert (st["trace_rays"], st["shadow_rays"]) == (cnt["trace_rays"], cnt["shadow_rays"])
