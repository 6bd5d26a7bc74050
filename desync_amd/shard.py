"""Multi-GPU range sharding (one process per GPU) -- make.go's split-and-align
across ranks.

Reference: IndexFromFile starts n workers span*i apart (make.go:69-116); each
chunks speculatively from its start and the main routine aligns it with its
predecessor when both produce the same chunk (syncWith, make.go:277-298).
Here rank r chunks [r*span, (r+1)*span) on its own GPU (dsx_shard_local),
the ranks all-gather fixed-size seam records (a few KB: the first candidates
and speculative cuts of each shard; RCCL over xGMI when the group uses the
"nccl" backend), and every rank aligns all seams (dsx_shard_resolve) to get
its exact slice of the sequential cut list.  The collective moves only seam
metadata, never blob bytes.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

SEAM_BYTES = ctypes.sizeof(_lib.Seam)


def seam_to_bytes(seam: "_lib.Seam") -> bytes:
    return ctypes.string_at(ctypes.addressof(seam), SEAM_BYTES)


def seams_from_bytes(blob: bytes, nranks: int):
    return (_lib.Seam * nranks).from_buffer_copy(blob)


def exchange_seams(seam_bytes: bytes, group=None, device=None) -> bytes:
    """All-gather one fixed-size seam record per rank (rank order)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    mine = torch.frombuffer(bytearray(seam_bytes), dtype=torch.uint8)
    if device is not None:
        mine = mine.to(device)
    bufs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(bufs, mine, group=group)
    return b"".join(b.cpu().numpy().tobytes() for b in bufs)


def shard_chunk(d_ptr, halo, shard_start, shard_len, total, params, ctx=None, group=None,
                device=None):
    """This rank's exact cut list (np.uint64 chunk end offsets c with
    shard_start < c <= shard_start + shard_len)."""
    import torch.distributed as dist
    ctx = ctx or _lib.default_context()
    seam = _lib.Seam()
    check(lib().dsx_shard_local(ctx.h, ctypes.c_void_p(d_ptr), halo, shard_start, shard_len,
                                total, ctypes.byref(params.c), ctypes.byref(seam)), ctx.h)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    allb = exchange_seams(seam_to_bytes(seam), group, device)
    arr = seams_from_bytes(allb, world)
    cap = shard_len // params.min + 4
    out = np.empty(cap, dtype=np.uint64)
    n = ctypes.c_uint64()
    check(lib().dsx_shard_resolve(ctx.h, arr, world, rank, out.ctypes.data, cap, ctypes.byref(n),
                                  0), ctx.h)
    return out[:n.value].copy()
