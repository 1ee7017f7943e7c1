"""Control experiment for the parity failures seen only when 8+ processes share one GPU
(DESIGN.md §2): N processes each repeat long-running GPU work (fp64 GEMMs of 2048^2, a few
ms each, and a long elementwise chain) on fixed inputs and compare every result bit for bit
with the first one computed in that process.  Uses torch only (no librtamd).

usage: python tools/gpu_share_check.py [procs] [rounds]"""
import multiprocessing as mp
import sys


def worker(k, rounds, q):
    import torch
    g = torch.Generator(device="cpu").manual_seed(1234 + k)
    a = torch.randn(2048, 2048, generator=g, dtype=torch.float64).cuda()
    b = torch.randn(2048, 2048, generator=g, dtype=torch.float64).cuda()
    v = torch.randn(1 << 22, generator=g, dtype=torch.float64).cuda()

    def work():
        c = a @ b
        w = v
        for _ in range(20):
            w = torch.sin(w) * 1.0001 + torch.sqrt(torch.abs(w))
        return c.cpu(), w.cpu()

    c0, w0 = work()
    bad = 0
    for r in range(rounds):
        c, w = work()
        bad += int((c.view(torch.int64) != c0.view(torch.int64)).sum()) + int((w.view(torch.int64) != w0.view(torch.int64)).sum())
    q.put((k, bad))


if __name__ == "__main__":
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(k, rounds, q)) for k in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    print({"procs": procs, "rounds": rounds, "mismatching_values": sum(b for _, b in res), "per_proc": sorted(res)})
