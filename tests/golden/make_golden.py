"""Generates tests/golden/ref_hashes.json from the UNMODIFIED reference.

Runs oracle/_ref/refharness (the reference's scene/geometry/parser sources compiled
where they lie under /root/reference by `make -C oracle ref`; see oracle/ref_harness.cpp)
over every parity case of tests/cases.py and records, per case:
  sha256 of the f64 RasterImage (little-endian, row-major H x W x 3),
  sha256 of the RGB8 bytes (writers.cpp:4-9 conversion),
  or the exit status + stderr for scenes the reference rejects.
It also records the shipped outputs/*.png SHA-256 and the config-size hashes.
Container-only (needs /root/reference); the JSON is the committed fixture.

    python tests/golden/make_golden.py [--configs]
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cases import CONFIGS, OPTION_SETS, REPO, SCENES, SHIPPED, scene_files  # noqa: E402

HARNESS = os.path.join(REPO, "oracle", "_ref", "refharness")
OUT = os.path.join(REPO, "tests", "golden", "ref_hashes.json")


def rgb8(raw):
    v = np.minimum(raw, 1.0)
    v = np.maximum(v, 0.0) * 255.0
    v = np.where(np.isnan(v), 0.0, v)
    return v.astype(np.uint8)


def run(scene, w, h, flags, threads=8):
    with tempfile.NamedTemporaryFile(suffix=".raw", delete=False) as tf:
        path = tf.name
    try:
        p = subprocess.run([HARNESS, scene, "-o", path, "-w", str(w), "-h", str(h), "-t", str(threads)] + flags,
                           cwd=SCENES, capture_output=True, text=True)
        if p.returncode:
            return {"rc": p.returncode, "stderr": p.stderr.strip().splitlines()[-1] if p.stderr.strip() else ""}
        raw = np.fromfile(path, dtype="<f8")
        return {"rc": 0, "f64_sha256": hashlib.sha256(raw.tobytes()).hexdigest(),
                "rgb8_sha256": hashlib.sha256(rgb8(raw).tobytes()).hexdigest()}
    finally:
        os.unlink(path)


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    data["generator"] = "tests/golden/make_golden.py via oracle/_ref/refharness (unmodified reference sources)"
    cases = {}
    for scene in scene_files():
        for name, w, h, flags in OPTION_SETS:
            cases[f"{scene}|{name}"] = run(scene, w, h, flags)
    data["cases"] = cases
    data["shipped_png_sha256"] = {
        k: hashlib.sha256(open(os.path.join(REPO, "tests", "golden", "shipped", k), "rb").read()).hexdigest()
        for k in SHIPPED}
    if "--configs" in sys.argv:
        cfg = {}
        for name, (scene, w, h, flags) in CONFIGS.items():
            cfg[name] = run(scene, w, h, flags)
            print(name, cfg[name], flush=True)
        data["configs"] = cfg
    json.dump(data, open(OUT, "w"), indent=1, sort_keys=True)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()
