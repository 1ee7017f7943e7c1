"""Phase profile of the traversal kernels on C3 (diagnostic; needs a librtamd built with
EXTRA_DEFS=-DRT_PHASE_PROF=1).  Per kernel variant: where the lanes' shader-clock cycles go
(sums over lanes of the wave's s_memtime deltas while the lane was active).

usage: RTAMD_LIB=cs184-raytracer_amd/rtamd/librtamd_prof.so python tools/phase_profile.py [frames]
(make -C cs184-raytracer_amd prof builds it)

Caveat: the shares are lane-weighted and the clock reads perturb scheduling; a phase that
ends with a memory wait can absorb latency that belongs to later work.  Timing-only
builds that skip a part ("Where the time goes") are the reliable check:
e.g. this tool put ~70 % of the level-0 k_shadow in its setup, while skipping the bunny's
LBVH showed the setup to be ~7 %."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from cases import CONFIGS, SCENES, option_kwargs  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = sys.argv[2] if len(sys.argv) > 2 else "C3_bunny_1920x1080_bd4"
scene, w, h, flags = CONFIGS[cfg]
kw = option_kwargs(flags)
s = rtamd.load_scene(os.path.join(SCENES, scene))
L = rtamd.lib()
L.rt_debug_phase_profile.restype = ctypes.c_int
L.rt_debug_phase_profile.argtypes = [ctypes.c_int, ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 32)()
out = torch.empty((h, w, 3), dtype=torch.float64, device="cuda")
prm = s.params(w, h, kw["bdepth"], False)
s.render_device(prm, out.data_ptr())
L.rt_debug_phase_profile(0, buf)  # clear after warm-up
for _ in range(frames):
    st = s.render_device(prm, out.data_ptr())
L.rt_debug_phase_profile(0, buf)
names = ["total", "nodes", "faces", "xform", "sphere", "world", "setup", "gate"]
for v, kname in enumerate(["k_closest per-lane", "k_closest packet", "k_shadow per-lane", "k_shadow packet"]):
    row = [buf[v * 8 + k] / frames for k in range(8)]
    if not row[0]:
        continue
    rest = row[0] - sum(row[1:8])
    print(f"{kname:20s} total {row[0] / 1e9:7.3f} Gcyc/frame  " +
          "  ".join(f"{names[k]} {100 * row[k] / row[0]:4.1f}%" for k in range(1, 8)) + f"  other {100 * rest / row[0]:4.1f}%")
print("rays/frame", st.rays // frames if False else st.trace_rays, st.shadow_rays)
