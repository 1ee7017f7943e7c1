"""The multi-rank frame partition (rtamd.dist) with the HIP renderer on every rank.

Two ranks (world size 2, gloo: both ranks share the box's one GPU, and RCCL needs one
GPU per rank) each render their interleaved rows with librtamd and the frame is
assembled on rank 0 by rtamd.dist: render_frame (f64, --intersection-only normalised by
the all-reduced maximum, scene.cpp:50-58) and the bench's RGB8 row gather.  Results are
compared with the unmodified reference's goldens (sha256 of the f64 image).
"""
import hashlib
import os
import tempfile

import numpy as np
import pytest

from cases import OPTION_SETS, SCENES, option_kwargs

pytestmark = pytest.mark.gpu


def _free_port():
    """A rendezvous for init_process_group: a fresh FileStore path (no TCP port to race for
    with the other test workers)."""
    return os.path.join(tempfile.mkdtemp(prefix="rtamd_pg_"), "store")


def _worker(rank, world, port, scene, w, h, bdepth, io, q, block):
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd import dist as rd
    os.environ.update(HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        s = rtamd.load_scene(scene)

        def render_rows(rows):
            n = rtamd.selected_count(*rows)
            out = torch.empty((n, w, 3), dtype=torch.float64, device="cuda")
            st = s.render_device(s.params(w, h, bdepth, io, rows[0], rows[1], rows[2], row_block=rows[3]),
                                 out.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
            return out, st.intersection_max
        frame = rd.render_frame(render_rows, h, io, torch.device("cuda"), block=block)
        # RGB8 rows (bench.py's partition step): rendered on the device, gathered to rank 0
        rows = rd.rank_rows(h, rank, world, block=block)
        n_buf = max(rd.n_rows(h, k, world, block) for k in range(world))
        out8 = torch.zeros((n_buf, w, 3), dtype=torch.uint8, device="cuda")
        if not io:
            s.render_device(s.params(w, h, bdepth, io, rows[0], rows[1], rows[2], row_block=rows[3]), 0,
                            out8.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        frame8 = rd.gather_rows(out8, h, dst=0, block=block)
        if rank == 0:
            q.put((frame.cpu().numpy(), None if io else frame8.cpu().numpy()))
        s.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scene,opt,block", [("excess_inputs/bunny.rti", "w64h48", 1),
                                             ("excess_inputs/refraction3.rti", "w50h30_bd12", 1),
                                             ("inputs/input-02.rti", "w31h17_io", 1), ("inputs/input-09.rti", "w37h23_bd2", 1),
                                             ("excess_inputs/bunny.rti", "w64h48", 8),
                                             ("inputs/input-02.rti", "w31h17_io", 4)])
def test_two_ranks_hip_partition_matches_reference(gpu, golden, scene, opt, block):
    import torch.multiprocessing as mp
    name, w, h, flags = next(o for o in OPTION_SETS if o[0] == opt)
    kw = option_kwargs(flags)
    ref = golden["cases"][f"{scene}|{name}"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = os.path.join(SCENES, scene)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, w, h, kw["bdepth"], kw["intersection_only"], q, block))
             for r in range(2)]
    for p in procs:
        p.start()
    got, got8 = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == ref["f64_sha256"]
    if got8 is not None:
        assert hashlib.sha256(np.ascontiguousarray(got8).tobytes()).hexdigest() == ref["rgb8_sha256"]
