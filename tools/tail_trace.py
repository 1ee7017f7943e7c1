"""Renders 1/N of the C3 frame (every N-th row, default 8) a few times; run it under
rocprofv3 --kernel-trace to see the fixed per-frame latency of the level chain
(tools/frame_timeline.py)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import rtamd  # noqa: E402
from cases import SCENES  # noqa: E402

s = rtamd.load_scene(os.path.join(SCENES, "excess_inputs/bunny.rti"))
s.upload()
W, H = 1920, 1080
step = int(sys.argv[1]) if len(sys.argv) > 1 else 8
out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
out8 = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
prm = s.params(W, H, 4, False, 0, H, step)
for _ in range(4):
    s.render_device(prm, out.data_ptr(), out8.data_ptr())
torch.cuda.synchronize()
