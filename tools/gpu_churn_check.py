"""Control experiment for the multi-process parity failures, torch only
(no librtamd): N processes each repeat, per iteration, the memory pattern of one small
fuzz render -- device buffers freshly allocated (the caching allocator emptied first, so
they are returned to and taken from the driver), a pinned host buffer allocated, a small
"record" of indices copied host-to-device on one stream, a gather kernel that reads it,
a second stream that writes a buffer the first stream then reads after an event, and a
device-to-host copy of the result -- and check every value against the same computation on
the CPU.

usage: python tools/gpu_churn_check.py [procs] [iterations]"""
import multiprocessing as mp
import sys


def worker(k, iters, q):
    import torch
    g = torch.Generator(device="cpu").manual_seed(4321 + k)
    main, side = torch.cuda.Stream(), torch.cuda.Stream()
    bad_iters = bad_values = 0
    first = None
    for it in range(iters):
        torch.cuda.empty_cache()
        n = int(torch.randint(2000, 40000, (1,), generator=g))
        src = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, dtype=torch.int64)
        idx = torch.randperm(n, generator=g)
        rec = idx.pin_memory()
        with torch.cuda.stream(main):
            d_src = torch.empty(n, dtype=torch.int64, device="cuda")
            d_src.copy_(src.pin_memory(), non_blocking=True)
            d_idx = torch.empty(n, dtype=torch.int64, device="cuda")
            d_idx.copy_(rec, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(main)
        with torch.cuda.stream(side):
            side.wait_event(ev)
            col = torch.abs(d_src) * 3 + 1  # the "shading" on the side stream (integer: exact)
            ev2 = torch.cuda.Event()
            ev2.record(side)
        with torch.cuda.stream(main):
            main.wait_event(ev2)
            out = col[d_idx] + d_src[d_idx]  # the "output" gather on the main stream
            host = torch.empty(n, dtype=torch.int64).pin_memory()
            host.copy_(out, non_blocking=True)
        main.synchronize()
        want = (torch.abs(src) * 3 + 1)[idx] + src[idx]
        nb = int((host != want).sum())
        if nb:
            bad_iters += 1
            bad_values += nb
            if first is None:
                first = (it, n, nb)
        del d_src, d_idx, col, out
    q.put((k, bad_iters, bad_values, first))


if __name__ == "__main__":
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(k, iters, q)) for k in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    print({"procs": procs, "iterations": iters, "bad_iterations": sum(r[1] for r in res),
           "bad_values": sum(r[2] for r in res), "per_proc": sorted(res)}, flush=True)
