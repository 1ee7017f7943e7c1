"""Frame-time scaling with the selected row fraction (tail-latency diagnostic): renders
1/1, 1/2, 1/4 and 1/8 of the C3 frame (row-interleaved) and prints ms and Mrays/s."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs184-raytracer_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch, rtamd
from cases import SCENES
s = rtamd.load_scene(os.path.join(SCENES, "excess_inputs/bunny.rti")); s.upload()
W, H = 1920, 1080
out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
out8 = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
for step in (1, 2, 4, 8):
    prm = s.params(W, H, 4, False, 0, H, step)
    for _ in range(3): s.render_device(prm, out.data_ptr(), out8.data_ptr())
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(10): st = s.render_device(prm, out.data_ptr(), out8.data_ptr())
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 10
    print(f"row step {step}: {dt*1e3:.3f} ms  rays {st.rays}  Mrays/s {st.rays/dt/1e6:.0f}")
