"""Multi-GPU frame partition for the render path: one process per GPU, RCCL over xGMI.

The reference renders one image with a thread pool over 2000-pixel blocks
(scene.cpp:13-48).  Here a frame is split into blocks of B rows (bench.py: B = 8, so the
8x8 ray tiles stay whole) interleaved over the ranks (row r is rendered by rank
(r // B) mod N: the costly glass/mirror regions of a frame are spread evenly),
each rank renders its rows on its own GPU (scene replicated in every GPU's HBM), and the
RGB8 rows are gathered to rank 0 — the only data-path exchange.  --intersection-only
needs one more collective: the reference normalises by the maximum over the whole image
(scene.cpp:50-58), so ranks all-reduce (MAX) their local maxima first.

The helpers take torch tensors (CUDA tensors with the "nccl" backend = RCCL, CPU tensors
with "gloo"), so the same code is exercised by the CPU tests.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def rank_rows(height: int, rank: int, world: int, shift: int = 0, block: int = 1) -> Tuple[int, int, int, int]:
    """(row_begin, row_end, row_step, row_block) of this rank's rows: blocks of `block` rows
    interleaved over the ranks (row r -> rank (r // block) mod world); with `shift`, rank r
    holds the blocks of residue (r + shift) mod world (frame `shift` of a rotated batch)."""
    return ((rank + shift) % world) * block, height, world, block


def rows_of(height: int, rank: int, world: int, block: int = 1):
    """The image rows of rank `rank`, in the order it renders them."""
    b = max(1, block)
    return [r for r in range(rank * b, height) if ((r - rank * b) // b) % world == 0]


def n_rows(height: int, rank: int, world: int, block: int = 1) -> int:
    return len(rows_of(height, rank, world, block))


def global_max(value: float, device: torch.device) -> float:
    """All-reduce MAX of a scalar (the --intersection-only normaliser)."""
    if dist.is_initialized() and dist.get_backend() == "gloo":
        device = torch.device("cpu")  # gloo reduces host tensors
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(local: torch.Tensor, height: int, dst: int = 0,
                out: Optional[torch.Tensor] = None, bufs: Optional[list] = None, shift: int = 0,
                group=None, group_size: Optional[int] = None,
                group_rank: Optional[int] = None, block: int = 1) -> Optional[torch.Tensor]:
    """Gathers every rank's interleaved rows (n_local, W, C) into a (H, W, C) frame on `dst`
    (rank r holds the row blocks of residue (r + shift) mod world, see rank_rows).  `local`
    may be longer than the rank's row count (a buffer of the longest rank's rows): the extra
    rows are ignored.  With `group` (a sub-communicator of ranks 0 .. group_size - 1),
    world = group_size and the rank is group_rank; `dst` is a global rank inside the group."""
    world = group_size if group is not None else (dist.get_world_size() if dist.is_initialized() else 1)
    rank = group_rank if group is not None else (dist.get_rank() if dist.is_initialized() else 0)
    if world == 1:
        rows = local[: height]
        if out is None:
            return rows.clone()
        out.copy_(rows)
        return out
    n_max = max(n_rows(height, k, world, block) for k in range(world))
    if not local.is_contiguous():
        local = local.contiguous()
    if local.shape[0] != n_max:
        pad = torch.zeros((n_max,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        k = min(n_max, local.shape[0])
        pad[:k] = local[:k]
        local = pad
    staged = local.is_cuda and dist.get_backend(group) == "gloo"  # gloo gathers host tensors
    if staged:
        local = local.cpu()
    if rank == dst:
        if bufs is None or staged:
            bufs = [torch.empty_like(local) for _ in range(world)]
        dist.gather(local, bufs, dst=dst, group=group)
        if out is None:
            out = torch.empty((height,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        for r in range(world):
            k = (r + shift) % world
            if block <= 1:
                out[k::world] = bufs[r][: n_rows(height, k, world)].to(out.device)
            else:
                idx = _row_index(height, k, world, block, out.device)
                out[idx] = bufs[r][: idx.numel()].to(out.device)
        return out
    dist.gather(local, None, dst=dst, group=group)
    return None


def band_rows(height: int, world: int, tile: int = 8) -> int:
    """Rows of one band when a frame is cut into `world` contiguous bands of whole 8-row ray
    tiles (the last band takes the rest): the block size of the multi-frame partition."""
    return max(tile, -(-height // (world * tile)) * tile)


def batch_rows(height: int, rank: int, world: int, frames: int, block: int = 1, rotate: bool = True):
    """This rank's row selection (rank_rows) of each of `frames` frames of one step.  rotate:
    frame f's share is the blocks of residue (rank + f) mod world (a rotated batch): over any
    `world` consecutive frames every rank renders every block of the image once, so with a
    step of a multiple of `world` frames of one scene the ranks' work is equal whatever the
    image's cost layout (the reference balances with its dynamic 2000-pixel block dispenser,
    scene.cpp:13-24; here the assignment is static, deterministic and known to the gather).
    With block = band_rows(height, world) each share is one contiguous band of the frame: the
    rows a GPU traces at once lie together in the image (L2 locality of the scene), and the
    rotation balances the bands' unequal costs over the step."""
    return [rank_rows(height, rank, world, shift=(f % world) if rotate else 0, block=block) for f in range(frames)]


def batch_order(rank: int, world: int, frames: int) -> list:
    """The order in which a rank hands its frames of a rotated batch (batch_rows) to one
    rt_render_batch_device call: within each cycle of `world` frames, by the residue of the
    blocks the rank renders, so that every rank's chunks hold the image's blocks in the same
    order (0, 1, ..., world - 1) and take the same time.  (Each frame keeps its own output
    rows, so the order changes neither the images nor the gather; measured: with frames in
    step order the ranks whose chunks start mid-image were up to 20% slower, bench.py
    --sweep, profiles/round6/ab/README.md.)"""
    order = []
    for c in range(0, frames, world):
        cyc = [f for f in range(c, min(c + world, frames))]
        order += sorted(cyc, key=lambda f: (rank + f) % world)
    return order


def gather_rows_batch(local: torch.Tensor, height: int, dst: int = 0, out: Optional[torch.Tensor] = None,
                      bufs: Optional[torch.Tensor] = None, block: int = 1,
                      rotate: bool = False) -> Optional[torch.Tensor]:
    """A batch of frames in ONE collective: `local` (F, n_buf, W, C) holds this rank's rows
    of F frames (n_buf >= its row count); on `dst`, out (F, H, W, C) receives every frame
    assembled from all ranks' rows (row blocks of `block` rows, see rank_rows; rotate: frame
    f's rows of rank r are the blocks of residue (r + f) mod world, see batch_rows).  bufs: a
    (world, F, n_buf, W, C) receive buffer on `dst` (made here when None).  The assembly is
    one gather (index_select) over a precomputed row map, not a copy per rank and frame."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if world == 1:
        if out is not None:
            out.copy_(local[:, :height])
        return out
    staged = local.is_cuda and dist.get_backend() == "gloo"
    src = local.cpu() if staged else local.contiguous()
    if rank == dst:
        shape = (world,) + tuple(src.shape)
        if bufs is None or staged or tuple(bufs.shape) != shape:
            bufs = torch.empty(shape, dtype=src.dtype, device=src.device)
        dist.gather(src, list(bufs.unbind(0)), dst=dst)
        F, n_buf = src.shape[0], src.shape[1]
        if out is None:
            out = torch.empty((F, height) + tuple(local.shape[2:]), dtype=local.dtype, device=local.device)
        idx = _batch_index(F, height, world, block, n_buf, rotate, bufs.device)
        rows = torch.index_select(bufs.reshape(world * F * n_buf, -1), 0, idx)
        out.view(F * height, -1).copy_(rows)
        return out
    dist.gather(src, None, dst=dst)
    return None


_ROW_INDEX = {}


def _row_index(height, rank, world, block, device):
    key = (height, rank, world, block, str(device))
    if key not in _ROW_INDEX:
        _ROW_INDEX[key] = torch.tensor(rows_of(height, rank, world, block), dtype=torch.long, device=device)
    return _ROW_INDEX[key]


_BATCH_INDEX = {}


def _batch_index(F, height, world, block, n_buf, rotate, device):
    """Row map of an assembled batch: entry f * height + r is the row of the gathered
    (world, F, n_buf) buffer that holds image row r of frame f."""
    key = (F, height, world, block, n_buf, rotate, str(device))
    if key not in _BATCH_INDEX:
        idx = torch.empty(F * height, dtype=torch.long)
        for f in range(F):
            for r in range(world):
                k = (r + f) % world if rotate else r
                rows = torch.tensor(rows_of(height, k, world, block), dtype=torch.long)
                idx[f * height + rows] = (r * F + f) * n_buf + torch.arange(rows.numel())
        _BATCH_INDEX[key] = idx.to(device)
    return _BATCH_INDEX[key]


def gather_frames(frame: torch.Tensor, dst: int = 0, out: Optional[list] = None) -> Optional[list]:
    """Frame-parallel mode: every rank's whole frame to `dst` (out[r] = rank r's frame)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if world == 1:
        if out is not None:
            out[0].copy_(frame)
        return out
    staged = frame.is_cuda and dist.get_backend() == "gloo"
    src = frame.cpu() if staged else frame.contiguous()
    if rank == dst:
        bufs = [torch.empty_like(src) for _ in range(world)] if staged or out is None else list(out)
        dist.gather(src, bufs, dst=dst)
        if out is not None and staged:
            for r in range(world):
                out[r].copy_(bufs[r])
        return out if out is not None else bufs
    dist.gather(src, None, dst=dst)
    return None


def gather_batch(full: torch.Tensor, height: int, dst: int = 0, frames: Optional[list] = None,
                 bufs: Optional[list] = None) -> Optional[list]:
    """A batch of `world` frames of one scene, each row-interleaved over all ranks.

    Frame f's rows of residue k mod world are rendered by rank (k - f) mod world, so over
    the batch every rank renders each row once: `full` (H, W, C) is this rank's single
    render of all rows, and frame f is assembled on `dst` from the rows every rank holds
    for it (one gather per frame).  Returns the frames on `dst`."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    outs = []
    for f in range(world):
        first = (rank + f) % world
        out = frames[f] if frames is not None and rank == dst else None
        outs.append(gather_rows(full[first::world], height, dst, out=out, bufs=bufs, shift=f))
    return outs if rank == dst else None


def render_frame(render_rows: Callable[[Tuple[int, int, int, int]], Tuple[torch.Tensor, float]], height: int,
                 intersection_only: bool, device: torch.device, dst: int = 0, block: int = 1) -> Optional[torch.Tensor]:
    """Distributed Scene::renderScene: returns the (H, W, 3) float64 frame on `dst`.

    render_rows(rows) renders this rank's rows (begin, end, step, block) and returns
    (float64 (n_local, W, 3), local max).  As rt_render/rt_render_device do, it returns
    --intersection-only values raw for a share of the rows and normalised for the whole
    image: one rank (world 1) selects every row, so its image is already final.
    """
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    img, local_max = render_rows(rank_rows(height, rank, world, block=block))
    if intersection_only and world > 1:
        m = global_max(max(local_max, 2.2250738585072014e-308), device)  # max init DBL_MIN (scene.cpp:51)
        img.mul_(1.0 / m)  # Color3d /= scalar multiplies by the reciprocal
    return gather_rows(img, height, dst, block=block)
