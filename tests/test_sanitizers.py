"""Sanitizer builds of the host C++ (race detection on the CPU build).

- ASan + UBSan over the product's host code: .rti/.obj ingest, flattening and LBVH build,
  PNG encoder (tests/native/host_check.cpp over every shipped scene);
- ASan + UBSan over the CPU oracle (its renders equal the normal build's);
- ThreadSanitizer over the oracle's 2000-pixel block threads (scene.cpp:13-48) and the
  same-algorithm CPU baseline's threads (oracle/cpu_bvh.cpp).  The reference itself races
  on its lazily transformed camera/lights; here every transform is
  computed once on the host, so no report may appear.
The GPU is not involved (GPU sanitizers are not available on the MI355X pool).
"""
import os
import subprocess

import numpy as np
import pytest

from cases import REPO, SCENES, scene_files

PKG = os.path.join(REPO, "cs184-raytracer_amd", "csrc")
ORACLE = os.path.join(REPO, "oracle")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
BASE = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-ffp-contract=off"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
           TSAN_OPTIONS="halt_on_error=1:exitcode=66")


def _build(out, srcs, flags):
    subprocess.run(BASE + flags + ["-o", str(out)] + srcs + ["-lz"], check=True, capture_output=True, timeout=600)


def test_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_check"
    _build(exe, [os.path.join(REPO, "tests", "native", "host_check.cpp")] +
           [os.path.join(PKG, f) for f in ("scene_host.cpp", "bvh.cpp", "png.cpp")], SAN)
    scenes = [os.path.join(SCENES, s) for s in scene_files()]
    p = subprocess.run([str(exe)] + scenes, capture_output=True, text=True, timeout=600, env=ENV)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
    assert p.stdout.strip().splitlines()[-1].startswith(f"ok {len(scenes) - 2} scenes, 2 rejected")


@pytest.fixture(scope="module")
def oracle_asan(tmp_path_factory):
    exe = tmp_path_factory.mktemp("asan") / "oracle_cli"
    _build(exe, [os.path.join(ORACLE, "oracle_cli.cpp"), os.path.join(ORACLE, "oracle.cpp")], SAN)
    return exe


@pytest.mark.parametrize("scene,flags", [("inputs/input-02.rti", ["--bdepth", "3"]), ("inputs/input-09.rti", []),
                                         ("excess_inputs/refraction3.rti", ["--bdepth", "8"]),
                                         ("inputs/input-03.rti", ["--intersection-only"])])
def test_oracle_under_asan_ubsan(oracle, oracle_asan, tmp_path, scene, flags):
    out = tmp_path / "img.raw"
    path = os.path.join(SCENES, scene)
    p = subprocess.run([str(oracle_asan), path, "-w", "36", "-h", "24", "-t", "4", "-o", str(out)] + flags,
                       capture_output=True, text=True, timeout=600, env=ENV)
    assert p.returncode == 0, p.stderr[-4000:]
    got = np.fromfile(out, dtype=np.float64).reshape(24, 36, 3)
    kw = {"bdepth": int(flags[1])} if flags[:1] == ["--bdepth"] else {}
    want, _ = oracle.render(path, 36, 24, intersection_only="--intersection-only" in flags, **kw)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_oracle_threads_under_tsan(tmp_path):
    exe = tmp_path / "oracle_tsan"
    _build(exe, [os.path.join(ORACLE, "oracle_cli.cpp"), os.path.join(ORACLE, "oracle.cpp")], ["-fsanitize=thread"])
    for scene in ("inputs/input-02.rti", "excess_inputs/refraction3.rti"):
        p = subprocess.run([str(exe), os.path.join(SCENES, scene), "-w", "60", "-h", "40", "-t", "8", "--bdepth", "4"],
                           capture_output=True, text=True, timeout=600, env=ENV)
        assert p.returncode == 0 and "ThreadSanitizer" not in p.stderr, p.stderr[-4000:]


def test_cpu_bvh_threads_under_tsan(tmp_path):
    exe = tmp_path / "cpu_bvh_tsan"
    _build(exe, [os.path.join(ORACLE, "cpu_bvh.cpp"), os.path.join(PKG, "scene_host.cpp"), os.path.join(PKG, "bvh.cpp")],
           ["-fsanitize=thread"])
    p = subprocess.run([str(exe), os.path.join(SCENES, "excess_inputs/bunny.rti"), "64", "36", "4", "8", "0", "36", "1",
                        "/dev/null"], capture_output=True, text=True, timeout=600, env=ENV)
    assert p.returncode == 0 and "ThreadSanitizer" not in p.stderr, p.stderr[-4000:]
