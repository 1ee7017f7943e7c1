"""BASELINE.json workloads: name -> (scene, width, height, reference flags).

Scenes are the reference's own inputs (copied under scenes/) plus the two authored config
scenes of SURVEY.md App. B (bunny.rti for C3, minicooper_sub.rti for C4).
"""
import os

SCENES = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "scenes")

CONFIGS = {
    "C1_simple_sphere_256": ("excess_inputs/simple_sphere.rti", 256, 256, []),
    "C2a_input01_1024_bd0": ("inputs/input-01.rti", 1024, 1024, ["--bdepth", "0"]),
    "C2b_input02_teapot_1024_bd0": ("inputs/input-02.rti", 1024, 1024, ["--bdepth", "0"]),
    "C3_bunny_1920x1080_bd4": ("excess_inputs/bunny.rti", 1920, 1080, ["--bdepth", "4"]),
    "C4_airboat_sub_1920x1080": ("excess_inputs/minicooper_sub.rti", 1920, 1080, []),
    "C5_refraction3_4096_bd8": ("excess_inputs/refraction3.rti", 4096, 4096, ["--bdepth", "8"]),
}


def option_kwargs(flags):
    """Reference flags (options.cpp:7-16) -> bdepth / intersection_only (defaults options.h:15-16)."""
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
