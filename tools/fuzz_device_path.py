"""The production-schedule fuzz scenes (tests/test_gpu_fuzz.py random_scene) rendered through
rt_render_device into device buffers (no host image path), by N processes sharing the GPU at
once, each against the CPU oracle: counts the seeds whose image differs (the
multi-process parity investigation).

usage: python tools/fuzz_device_path.py <procs> <base> <seeds>"""
import multiprocessing as mp
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(k, procs, base, seeds, q):
    sys.path[:0] = [os.path.join(REPO, "cs184-raytracer_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
    import pathlib
    import numpy as np
    import torch
    import pyoracle
    import rtamd
    from test_gpu_fuzz import random_scene
    bad = []
    done = 0
    for seed in range(base + k, base + seeds, procs):
        done += 1
        if done % 50 == 0:
            print(f"worker {k}: {done} seeds, {len(bad)} differ", flush=True)
        with tempfile.TemporaryDirectory() as d:
            path, bdepth, io = random_scene(seed, pathlib.Path(d))
            try:
                want, _ = pyoracle.render(path, 56, 40, bdepth=bdepth, intersection_only=io)
            except RuntimeError:
                continue
            s = rtamd.load_scene(path)
            out = torch.empty((40, 56, 3), dtype=torch.float64, device="cuda")
            ok = True
            for _ in range(2):
                s.render_device(s.params(56, 40, bdepth, io), out.data_ptr())
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                ok = ok and np.array_equal(got.view(np.uint64), want.view(np.uint64))
            s.close()
            if not ok:
                bad.append(seed)
    q.put((k, bad))


if __name__ == "__main__":
    procs, base, seeds = (int(v) for v in sys.argv[1:4])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(k, procs, base, seeds, q)) for k in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    bad = sorted(s for _, b in res for s in b)
    print({"procs": procs, "seeds": seeds, "failed": len(bad), "failed_seeds": bad[:20]})
