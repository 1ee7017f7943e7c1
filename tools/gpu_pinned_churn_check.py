"""Control experiment for the multi-process parity failures, torch plus
the HIP runtime through ctypes (no librtamd): N processes each keep S streams busy, and every
round every stream gets a freshly allocated device buffer filled by an asynchronous
hipMemcpyAsync from a pinned host buffer that was itself just allocated with hipHostMalloc
and is freed right after (the allocation churn of a librtamd scene: pinned staging, row
tables and level records per scene).  Every result is compared with the CPU.

usage: python tools/gpu_pinned_churn_check.py [procs] [streams] [rounds]"""
import ctypes
import multiprocessing as mp
import sys


def worker(k, n_streams, rounds, q):
    import numpy as np
    import torch
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    rng = np.random.default_rng(99 + k)
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    bad = 0
    for r in range(rounds):
        torch.cuda.empty_cache()
        jobs = []
        for s in streams:
            n = int(rng.integers(1000, 200000))
            src = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
            pin = ctypes.c_void_p()
            assert hip.hipHostMalloc(ctypes.byref(pin), n * 8, 0) == 0
            np.ctypeslib.as_array((ctypes.c_int64 * n).from_address(pin.value))[:] = src
            with torch.cuda.stream(s):
                d = torch.empty(n, dtype=torch.int64, device="cuda")
                assert hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), pin, n * 8, 1, ctypes.c_void_p(s.cuda_stream)) == 0
                y = (d * 3 + 7) ^ (d >> 5)
            jobs.append((s, pin, src, y))
        for s, pin, src, y in jobs:
            s.synchronize()
            hip.hipHostFree(pin)
            want = (src * 3 + 7) ^ (src >> 5)
            bad += int((y.cpu().numpy() != want).sum())
        if k == 0 and r % 100 == 0:
            print(f"worker 0 round {r}", flush=True)
    q.put((k, bad))


if __name__ == "__main__":
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n_streams = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(k, n_streams, rounds, q)) for k in range(procs)]
    for p in ps:
        p.start()
    res = []
    for _ in ps:
        try:
            res.append(q.get(timeout=600))
        except Exception:  # a worker died (e.g. a GPU memory fault): report its exit code
            break
    for p in ps:
        p.join(timeout=30)
    print({"procs": procs, "streams": n_streams, "rounds": rounds, "mismatching_values": sum(b for _, b in res),
           "per_proc": sorted(res), "exit_codes": [p.exitcode for p in ps]}, flush=True)
