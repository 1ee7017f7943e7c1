"""Lane occupancy census of the per-lane kernels on C3 (diagnostic build with
-DRT_DIAG_LANES=1: tools/build_variant.sh lanes -DRT_DIAG_LANES=1).

usage: RTAMD_LIB=cs184-raytracer_amd/rtamd/var/librtamd_lanes.so python tools/lane_census.py [frames]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd.configs import CONFIGS, SCENES, option_kwargs  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = sys.argv[2] if len(sys.argv) > 2 else "C3_bunny_1920x1080_bd4"
scene, w, h, flags = CONFIGS[cfg]
kw = option_kwargs(flags)
s = rtamd.load_scene(os.path.join(SCENES, scene))
s.upload()
L = rtamd.lib()
L.rt_debug_phase_profile.restype = ctypes.c_int
L.rt_debug_phase_profile.argtypes = [ctypes.c_int, ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 32)()
out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
prm = s.params(w, h, kw["bdepth"], False)
s.render_device(prm, out.data_ptr())
L.rt_debug_phase_profile(0, buf)  # clear after warm-up
for _ in range(frames):
    s.render_device(prm, out.data_ptr())
L.rt_debug_phase_profile(0, buf)
rows = [(0, "k_closest<false>: active lanes per wave slot"),
        (2, "k_closest<false>: lanes in the geometry loop per iteration"),
        (4, "k_closest<false>: lanes entering a geometry (world box hit) per iteration"),
        (6, "k_closest<false>: iterations in which some lane enters the geometry"),
        (14, "k_closest<false>: lanes in a linear face test"),
        (12, "k_shadow<false>: lanes in a linear face test"),
        (20, "k_shadow<false>: lanes still searching per geometry iteration"),
        (22, "k_shadow<false>: lanes entering a geometry (world box hit) per iteration"),
        (30, "k_shadow<false>: iterations in which some lane enters the geometry"),
        (28, "k_shadow<false>: lanes shading in place (per-lane fused Phong)"),
        (8, "k_closest<false>: lanes entering an LBVH search per wave entering"),
        (10, "k_closest<false>: lanes holding a leaf per face phase"),
        (16, "k_shadow<false>: lanes with a hit per wave slot"),
        (18, "k_shadow<false>: lanes tracing (not zero-term) per wave slot"),
        (24, "k_shadow<false>: lanes entering an LBVH search per wave entering"),
        (26, "k_shadow<false>: lanes holding a leaf per face phase")]
for k, what in ([] if os.environ.get("RTAMD_DIAG_GEOMS") else rows):
    slots, lanes = buf[k], buf[k + 1]
    if slots:
        print(f"{what:70s} {lanes / slots:6.3f}  ({slots / 64 / frames:12.0f} wave events/frame)")
# RT_DIAG_GEOMS builds: per shadow-order position, packet shadow waves with candidates
if os.environ.get("RTAMD_DIAG_GEOMS"):
    for k in range(16):
        if buf[2 * k]:
            print(f"packet shadow, shadow-order position {k}: {buf[2 * k] / 64 / frames:10.0f} waves/frame with "
                  f"candidates, {buf[2 * k + 1] / buf[2 * k]:.3f} of their lanes")
s.close()
