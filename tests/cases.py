"""Parity cases shared by the golden generator (tests/golden/make_golden.py) and the tests.

Scenes are the reference's own inputs (inputs/*.rti, excess_inputs/*.rti, data files
copied under scenes/) plus the two authored config scenes of SURVEY.md App. B.
"""
import glob
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")


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


def option_kwargs(flags):
    bdepth, io = 10, False
    i = 0
    while i < len(flags):
        if flags[i] == "--bdepth":
            bdepth = int(flags[i + 1])
            i += 2
        elif flags[i] == "--intersection-only":
            io = True
            i += 1
        else:
            raise ValueError(flags[i])
    return {"bdepth": bdepth, "intersection_only": io}


# BASELINE.json configs: name -> (scene, W, H, flags)
CONFIGS = {
    "C1_simple_sphere_256": ("excess_inputs/simple_sphere.rti", 256, 256, []),
    "C2a_input01_1024_bd0": ("inputs/input-01.rti", 1024, 1024, ["--bdepth", "0"]),
    "C2b_input02_teapot_1024_bd0": ("inputs/input-02.rti", 1024, 1024, ["--bdepth", "0"]),
    "C3_bunny_1920x1080_bd4": ("excess_inputs/bunny.rti", 1920, 1080, ["--bdepth", "4"]),
    "C4_airboat_sub_1920x1080": ("excess_inputs/minicooper_sub.rti", 1920, 1080, []),
    "C5_refraction3_4096_bd8": ("excess_inputs/refraction3.rti", 4096, 4096, ["--bdepth", "8"]),
}

# The reference's shipped renders (outputs/image-0N.png, notes/notes-0N.txt:3)
SHIPPED = {f"image-0{i}.png": (f"inputs/input-0{i}.rti", 2000 if i == 9 else 1000, 2000 if i == 9 else 1000)
           for i in range(1, 10)}
