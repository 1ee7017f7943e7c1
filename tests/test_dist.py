"""Row-interleaved multi-rank partition + gather (rtamd.dist), world_size 2 over gloo on CPU.

The per-rank renderer here is the CPU oracle (test infrastructure); on GPUs the same
rtamd.dist code runs with the "nccl" (RCCL) backend and the HIP renderer (bench.py).
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from cases import SCENES


def _free_port():
    """A rendezvous for init_process_group: a fresh FileStore path (no TCP port to race for
    with the other test workers)."""
    return os.path.join(tempfile.mkdtemp(prefix="rtamd_pg_"), "store")


def _worker(rank, world, port, scene, w, h, bdepth, io, q, block=1):
    import torch.distributed as dist
    import pyoracle
    from rtamd import dist as rd
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        def render_rows(rows):
            begin, end, step, block = rows
            if block == 1:
                img, _ = pyoracle.render(scene, w, h, bdepth=bdepth, intersection_only=io, threads=2,
                                         rows=(begin, end, step))
            else:  # row blocks: the oracle's full image, this rank's rows
                full, _ = pyoracle.render(scene, w, h, bdepth=bdepth, intersection_only=io, threads=2)
                img = np.ascontiguousarray(full[rd.rows_of(h, begin // block, step, block)])
            local_max = float(np.nanmax(img)) if img.size else 0.0
            return torch.from_numpy(img), local_max
        frame = rd.render_frame(render_rows, h, io, torch.device("cpu"), block=block)
        if rank == 0:
            q.put(frame.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scene,io,block", [("excess_inputs/refraction3.rti", False, 1), ("inputs/input-02.rti", True, 1),
                                            ("inputs/input-09.rti", False, 1), ("excess_inputs/refraction3.rti", False, 4),
                                            ("inputs/input-02.rti", True, 3)])
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_frame_equals_single_render(oracle, scene, io, block, world):
    w, h, bdepth = 33, 23, 4
    path = os.path.join(SCENES, scene)
    want, _ = oracle.render(path, w, h, bdepth=bdepth, intersection_only=io)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, w, h, bdepth, io, q, block)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(got, want)


def _batch_worker(rank, world, port, scene, w, h, bdepth, q):
    import torch.distributed as dist
    import pyoracle
    from rtamd import dist as rd
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        img, _ = pyoracle.render(scene, w, h, bdepth=bdepth, threads=2)
        full = torch.from_numpy(img)
        frames = rd.gather_batch(full, h)
        if rank == 0:
            q.put([fr.numpy() for fr in frames])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rotated_batch_assembles_every_frame(oracle, world):
    """bench.py's N-frame step: frame f's rows come from all ranks (rotated interleave)."""
    w, h, bdepth = 29, 17, 3
    path = os.path.join(SCENES, "excess_inputs/bunny.rti")
    want, _ = oracle.render(path, w, h, bdepth=bdepth)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, path, w, h, bdepth, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == world
    for fr in got:
        assert np.array_equal(fr, want)


def _batch_rows_worker(rank, world, port, scene, w, h, bdepth, block, q, rotate=False, frames=3):
    import torch.distributed as dist
    import pyoracle
    from rtamd import dist as rd
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        full, _ = pyoracle.render(scene, w, h, bdepth=bdepth, threads=2)
        n_buf = max(rd.n_rows(h, k, world, block) for k in range(world))
        local = torch.zeros((frames, n_buf, w, 3), dtype=torch.float64)
        work = 0
        for f, sel in enumerate(rd.batch_rows(h, rank, world, frames, block, rotate)):
            # frame f: the image scaled by f + 1, this rank's rows of it (the selection bench.py renders)
            rows = [r for r in range(sel[0], sel[1]) if ((r - sel[0]) // sel[3]) % sel[2] == 0]
            local[f, : len(rows)] = torch.from_numpy(full[rows] * (f + 1))
            work += len(rows)
        out = rd.gather_rows_batch(local, h, block=block, rotate=rotate)
        counts = [None] * world
        dist.all_gather_object(counts, work)
        if rank == 0:
            q.put((out.numpy(), counts))
    finally:
        dist.destroy_process_group()


def _run_batch_rows(oracle, world, block, rotate, frames):
    w, h, bdepth = 21, 29, 3
    path = os.path.join(SCENES, "excess_inputs/bunny.rti")
    want, _ = oracle.render(path, w, h, bdepth=bdepth)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_rows_worker, args=(r, world, port, path, w, h, bdepth, block, q, rotate, frames))
             for r in range(world)]
    for p in procs:
        p.start()
    got, counts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for f in range(frames):
        assert np.array_equal(got[f], want * (f + 1))
    return counts


@pytest.mark.parametrize("world,block", [(2, 8), (3, 4), (3, 1), (8, 8), (8, 1)])
def test_batched_row_gather(oracle, world, block):
    """bench.py's partition step: all frames of a step gathered in one collective and
    de-interleaved on rank 0 (row blocks)."""
    _run_batch_rows(oracle, world, block, False, 3)


@pytest.mark.parametrize("world,block,frames", [(2, 8, 4), (3, 4, 6), (8, 8, 16), (8, 1, 8), (8, 8, 3),
                                               (2, "band", 4), (3, "band", 3), (8, "band", 8)])
def test_rotated_batch_row_gather_balances_ranks(oracle, world, block, frames):
    """bench.py's partition step with the rotated assignment (rtamd.dist.batch_rows): frame
    f's blocks of residue (r + f) mod world go to rank r; the gather puts every row back
    exactly, and over a multiple of `world` frames every rank renders the same rows in
    total (the same work)."""
    if block == "band":  # bench.py's default: one contiguous band of whole 8-row tiles per rank
        from rtamd import dist as rd
        block = rd.band_rows(29, world)
    counts = _run_batch_rows(oracle, world, block, True, frames)
    if frames % world == 0:
        assert len(set(counts)) == 1, counts


@pytest.mark.parametrize("scene,io,block", [("excess_inputs/refraction3.rti", False, 8), ("inputs/input-02.rti", True, 1)])
def test_partitioned_frame_world8(oracle, scene, io, block):
    """The driver's 8-GPU layout (one rank per GPU of a node) over gloo: with 8-row blocks
    ranks 3-7 of a 23-row frame own no rows, and their empty shares still take part in the
    gather and in the --intersection-only all-reduce(MAX)."""
    test_partitioned_frame_equals_single_render(oracle, scene, io, block, 8)


@pytest.mark.parametrize("io", [False, True])
def test_single_rank_frame_is_the_single_render(oracle, io):
    """world 1 (no process group): the rank's selection is the whole image, which the
    renderer already normalised for --intersection-only; render_frame must not divide by
    the maximum a second time (dist.py)."""
    from rtamd import dist as rd
    import pyoracle
    w, h, bdepth = 31, 19, 3
    path = os.path.join(SCENES, "inputs/input-02.rti")
    want, _ = oracle.render(path, w, h, bdepth=bdepth, intersection_only=io)

    def render_rows(rows):
        begin, end, step, block = rows
        assert (begin, end, step) == (0, h, 1)
        img, _ = pyoracle.render(path, w, h, bdepth=bdepth, intersection_only=io, threads=2)
        # a renderer reports its raw maximum; here the image is normalised, so any value > 1
        # would expose a second normalisation
        return torch.from_numpy(img), 7.0
    frame = rd.render_frame(render_rows, h, io, torch.device("cpu"), block=8)
    assert np.array_equal(frame.numpy(), want)


@pytest.mark.parametrize("world,frames", [(1, 5), (2, 4), (3, 7), (8, 48), (8, 3)])
def test_batch_order_puts_every_rank_blocks_in_one_order(world, frames):
    """bench.py hands each rank's frames of a rotated batch to the batch call in
    rtamd.dist.batch_order: a permutation of the step's frames, cycle by cycle, under which
    every rank renders the image's blocks in the order 0, 1, ..., world - 1 (so all ranks'
    chunks hold the same block sequence)."""
    from rtamd import dist as rd
    for rank in range(world):
        order = rd.batch_order(rank, world, frames)
        assert sorted(order) == list(range(frames))
        for c in range(0, frames, world):
            cyc = order[c:c + world]
            assert sorted(cyc) == list(range(c, min(c + world, frames)))
            residues = [(rank + f) % world for f in cyc]
            assert residues == sorted(residues)
            if len(cyc) == world:
                assert residues == list(range(world))
