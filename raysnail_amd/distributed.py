"""Multi-GPU sharding of the render path: one process per GPU, torch.distributed (RCCL over xGMI
on MI355X, gloo in the CPU tests).

raysnail itself only splits rows over CPU threads (src/painter.rs:239-299: thread i renders rows
i, i+T, ... and Painter::append de-interleaves them). The GPU path keeps both of the reference's
natural shardings, each with a single exchange at frame end:

* ``rows``   — one frame, rows interleaved over ranks exactly like render_rows (row r on rank
               r % N); ranks pack their rows, gather them to rank 0 and it de-interleaves them
               (= append, painter.rs:220-236). Strong scaling; the assembled frame is bitwise
               equal to the 1-GPU frame because every sample has its own RNG stream.
* ``passes`` — the CLI's progressive passes (src/bin/raysnail.rs:379-427): rank r renders pass r
               of the whole frame; the N pass frames are gathered to rank 0 and folded in pass order with
               combine_pixel (raysnail.rs:176-208). Weak scaling: per-GPU work is one full pass.

The renderer is injected (``render(row_begin, row_end, row_step, pass_index) -> (H, W, 4)``), so
the same code runs over libraysnail_hip on the GPU and over the CPU oracle in the gloo tests.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


def row_lattice(rank: int, world: int):
    """Rows of rank `rank`: rank, rank + world, ... (painter.rs:248)."""
    return rank, 0, world


def rows_of(rank: int, world: int, height: int) -> int:
    return (height - rank + world - 1) // world if rank < height else 0


_ROWBUF = {}


def gather_rows(frame: torch.Tensor, rank: int, world: int, dst: int = 0):
    """frame: (H, W, 4) with this rank's lattice rows rendered. Each rank packs its rows and sends
    them to rank `dst` (one RCCL gather at frame end), which de-interleaves them (Painter::append,
    painter.rs:220-236). Returns the full frame on dst, None elsewhere.

    Per frame: one strided copy (pack), the gather straight into a (world, per, W, 4) buffer, and on
    dst one permuted copy into a (per * world, W, 4) frame whose rows p * world + r are rank r's p-th
    row (the rows past H are padding). The staging buffers of the last frame shape are kept across
    frames; the returned frame is a fresh tensor (a caller may keep it, e.g. to combine passes)."""
    H = frame.shape[0]
    if world == 1:
        return frame
    per = (H + world - 1) // world
    rest = tuple(frame.shape[1:])
    key = (rest, H, frame.dtype, frame.device, rank, world, dst)
    buf = _ROWBUF.get(key)
    if buf is None:
        packed = torch.zeros((per,) + rest, dtype=frame.dtype, device=frame.device)
        allp = torch.empty((world, per) + rest, dtype=frame.dtype, device=frame.device) if rank == dst else None
        _ROWBUF.clear()  # one shape's buffers at a time
        _ROWBUF[key] = buf = (packed, allp)
    packed, allp = buf
    n = rows_of(rank, world, H)
    packed[:n].copy_(frame[rank::world])
    dist.gather(packed, list(allp.unbind(0)) if rank == dst else None, dst=dst)
    if rank != dst:
        return None
    full = torch.empty((per * world,) + rest, dtype=frame.dtype, device=frame.device)
    full.view((per, world) + rest).copy_(allp.transpose(0, 1))
    return full[:H]


def combine_pixels(old: torch.Tensor, new: torch.Tensor, p: float) -> torch.Tensor:
    """raysnail.rs:176-208: keep old where new is [0,0,0,0], else (old*p + new)/(p+1), f32."""
    empty = (new == 0).all(dim=-1, keepdim=True)
    pp = torch.tensor(p, dtype=torch.float32, device=new.device)
    mixed = (old * pp + new) / (pp + 1.0)
    return torch.where(empty, old, mixed)


def gather_passes(frame: torch.Tensor, rank: int, world: int, dst: int = 0):
    """All ranks' pass frames -> rank `dst` folds them in pass order (starting from the CLI's
    initial [0,0,0,1] image, raysnail.rs:317-322). Returns the combined frame on dst, else None."""
    if world == 1:
        parts = [frame]
    else:
        parts = [torch.empty_like(frame) for _ in range(world)] if rank == dst else None
        dist.gather(frame, parts, dst=dst)
    if rank != dst:
        return None
    acc = torch.zeros_like(frame)
    acc[..., 3] = 1.0
    for p, f in enumerate(parts):
        acc = combine_pixels(acc, f, float(p))
    return acc


def render_sharded(render: Callable[[int, int, int, int], torch.Tensor], rank: int, world: int, split: str):
    """One frame step of the job. split = 'rows' (strong) or 'passes' (weak)."""
    if split == "rows":
        rb, re, rs = row_lattice(rank, world)
        return gather_rows(render(rb, re, rs, 0), rank, world)
    if split == "passes":
        return gather_passes(render(0, 0, 1, rank), rank, world)
    raise ValueError(split)
