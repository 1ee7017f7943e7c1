"""Wave census of the packet searches on a config, in the bench's batch schedule (diagnostic
build: tools/build_variant.sh pk -DRT_DIAG_PACKET=1; the counting perturbs timing, not counts).

Per frame: how many wave node iterations, face tests and face-test stages the packet
kernels run, and how many of their 64 lanes take part (intersect.h PacketSlot).

usage: RTAMD_LIB=cs184-raytracer_amd/rtamd/var/librtamd_pk.so python tools/packet_census.py [frames] [config]"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
os.environ.setdefault("RTAMD_SERIAL", "1")
os.environ.setdefault("RTAMD_BATCH_LANES", "1")
import torch  # noqa: E402
import rtamd  # noqa: E402
from rtamd.configs import CONFIGS, SCENES, option_kwargs  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = sys.argv[2] if len(sys.argv) > 2 else "C3_bunny_1920x1080_bd4"
scene, w, h, flags = CONFIGS[cfg]
kw = option_kwargs(flags)
s = rtamd.load_scene(os.path.join(SCENES, scene))
s.upload()
L = rtamd.lib()
L.rt_debug_phase_profile.restype = ctypes.c_int
L.rt_debug_phase_profile.argtypes = [ctypes.c_int, ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 32)()
outs = [torch.empty((h, w, 3), dtype=torch.float64, device="cuda") for _ in range(frames)]
prm = [s.params(w, h, kw["bdepth"], kw["intersection_only"], 0, h, 1)] * frames
stream = torch.cuda.current_stream().cuda_stream
s.render_batch_device(prm, [o.data_ptr() for o in outs], [], stream)
torch.cuda.synchronize()
L.rt_debug_phase_profile(0, buf)  # clear after the warm-up
st = s.render_batch_device(prm, [o.data_ptr() for o in outs], [], stream)
torch.cuda.synchronize()
L.rt_debug_phase_profile(0, buf)
names = ["shadow node iterations", "shadow face tests", "  past facing", "  past D/Da", "  past a/Db", "  past b/Dt",
         "  candidates", "shadow LBVH entries", "shadow geometries entered", "shadow light verdicts",
         "closest node iterations", "closest face tests", "  candidates", "closest LBVH entries",
         "closest geometries entered", "closest items"]
res = {}
for k, nm in enumerate(names):
    slots, lanes = buf[2 * k], buf[2 * k + 1]
    waves = slots / 64 / frames
    res[nm.strip()] = {"waves_per_frame": round(waves), "lanes_per_wave": round(lanes / slots, 3) if slots else None}
    print(f"{nm:28s} {waves:12.0f} wave events/frame   {lanes / slots if slots else 0:6.3f} of the lanes")
print(json.dumps({"config": cfg, "frames": frames, "shadow_rays": st.shadow_rays // frames, "census": res}))
s.close()
