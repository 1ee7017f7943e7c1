"""INTEGRATION.md §1 end to end (gpu): the binding that gives the reference's
Scene::renderScene (scene.cpp:10-59) its GPU body, compiled against the UNMODIFIED
reference classes (oracle/_ref/integration_check, `make -C oracle ref` in the container
that holds /root/reference; the binary travels to the GPU box with the tree).

One process parses each scene with the reference's own RTIParser/OBJParser, describes the
in-memory Scene to librtamd (rt_scene_create_desc), renders it on the GPU (rt_render) and
then runs the reference's own renderScene on the same Scene: the two RasterImages must be
identical binary64 for binary64.  W*H is a multiple of 2000 (the reference's block).
"""
import os
import subprocess

import pytest

from cases import REPO, SCENES, scene_files

pytestmark = pytest.mark.gpu

EXE = os.path.join(REPO, "oracle", "_ref", "integration_check")


def good_scenes(golden):
    return [s for s in scene_files() if golden["cases"][f"{s}|w64h48"]["rc"] == 0]


@pytest.mark.parametrize("flags", [[], ["--bdepth", "2"], ["--intersection-only"]], ids=["default", "bd2", "io"])
def test_reference_scene_render_on_gpu(golden, flags):
    if not os.access(EXE, os.X_OK):
        pytest.skip("oracle/_ref/integration_check not built (needs /root/reference at build time)")
    def run(scene):
        return scene, subprocess.run([EXE, os.path.join(SCENES, scene), "-o", "/dev/null", "-w", "80", "-h", "50"] +
                                     flags, capture_output=True, text=True, timeout=120)

    # one process on the card at a time (the round-5 multi-process records: DESIGN.md §2)
    results = [run(scene) for scene in good_scenes(golden)]
    bad = [(s, p.returncode, p.stdout.strip(), p.stderr.strip()[-200:]) for s, p in results
           if p.returncode != 0 or not p.stdout.startswith("match 4000")]
    assert not bad, bad
