"""Parity cases shared by the golden generator (tests/golden/make_golden.py) and the tests.

Scenes are the reference's own inputs (inputs/*.rti, excess_inputs/*.rti, data files
copied under scenes/) plus the two authored config scenes of SURVEY.md App. B.
"""
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))


def scene_files():
    """All .rti scenes, repo-relative ('inputs/input-01.rti', ...), sorted."""
    out = []
    for sub in ("inputs", "excess_inputs"):
        out += sorted(os.path.relpath(p, SCENES) for p in glob.glob(os.path.join(SCENES, sub, "*.rti")))
    return out


# (name, width, height, extra reference flags)
OPTION_SETS = [
    ("w64h48", 64, 48, []),
    ("w37h23_bd2", 37, 23, ["--bdepth", "2"]),
    ("w40h40_bd0", 40, 40, ["--bdepth", "0"]),
    ("w31h17_io", 31, 17, ["--intersection-only"]),
    ("w50h30_bd12", 50, 30, ["--bdepth", "12"]),
]


from rtamd.configs import CONFIGS, option_kwargs  # noqa: E402,F401  (BASELINE.json configs, shared with bench.py)


# The reference's shipped renders (outputs/image-0N.png, notes/notes-0N.txt:3)
SHIPPED = {f"image-0{i}.png": (f"inputs/input-0{i}.rti", 2000 if i == 9 else 1000, 2000 if i == 9 else 1000)
           for i in range(1, 10)}


# The suite runs the library's own (production) schedule.  Small test images make every
# shading launch of a single frame trace light-major (api.cpp light_major_below) and every
# replayed chunk issue on one stream (one_stream_pixels), so the all-lights, fused-Phong and
# multi-stream forms the full-size renders use are run explicitly where they matter: with
# ALL_FORMS (the `schedule` parametrisations: every shipped scene and option set, the fuzz
# sweep's even seeds, the knob tests).
ALL_FORMS = {"RTAMD_LIGHT_MAJOR_BELOW": "0", "RTAMD_ONE_STREAM_PIXELS": "0"}
SCHEDULES = ["production", "all-forms"]


def apply_schedule(monkeypatch, schedule):
    """`schedule`: "production" (the library's defaults) or "all-forms" (ALL_FORMS)."""
    for k, v in ALL_FORMS.items():
        if schedule == "all-forms":
            monkeypatch.setenv(k, v)
        else:
            monkeypatch.delenv(k, raising=False)
