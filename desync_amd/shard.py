"""Multi-GPU range sharding (one process per GPU) -- make.go's split-and-align
across ranks.

Reference: IndexFromFile starts n workers span*i apart (make.go:69-116); each
chunks speculatively from its start and the main routine aligns it with its
predecessor when both produce the same chunk (syncWith, make.go:277-298).
Here rank r chunks [r*span, (r+1)*span) on its own GPU (dsx_shard_local),
the ranks all-gather fixed-size seam records (16 KiB: the first candidates
and speculative cuts of each shard; RCCL over xGMI when the group uses the
"nccl" backend, the records never leave HBM), and every rank aligns all seams
(dsx_shard_resolve) to get its exact slice of the sequential cut list.  A
seam that does not converge inside its window (a zero run across a shard
boundary -- README.md:114-119) makes its owner re-walk its shard from the
true entry cut; the ranks then exchange the records again
(dsx_shard_resolve returns DSX_E_RESYNC; at most nranks rounds).  The
collective moves only seam metadata, never blob bytes.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import DSX_E_RESYNC, DSX_OUT_DEVICE, DSX_SEAM_DEVICE, check, lib

SEAM_BYTES = ctypes.sizeof(_lib.Seam)


def seam_to_bytes(seam: "_lib.Seam") -> bytes:
    return ctypes.string_at(ctypes.addressof(seam), SEAM_BYTES)


def seams_from_bytes(blob: bytes, nranks: int):
    return (_lib.Seam * nranks).from_buffer_copy(blob)


def exchange_seams(seam_bytes: bytes, group=None, device=None) -> bytes:
    """All-gather one fixed-size seam record per rank (rank order), host bytes."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    mine = torch.frombuffer(bytearray(seam_bytes), dtype=torch.uint8)
    if device is not None:
        mine = mine.to(device)
    bufs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(bufs, mine, group=group)
    return b"".join(b.cpu().numpy().tobytes() for b in bufs)


class DeviceShard:
    """The N>1 path with the seam records in HBM (RCCL all-gather in place).

    ``run()`` chunks this rank's shard and returns its exact cut count; the
    cuts stay in ``self.out`` (an int64 device tensor) -- the bench's step.
    """

    def __init__(self, ctx, d_ptr, halo, shard_start, shard_len, total, params, group=None):
        import torch
        import torch.distributed as dist
        self.ctx, self.d_ptr, self.halo = ctx, d_ptr, halo
        self.start, self.len, self.total, self.params = shard_start, shard_len, total, params
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = torch.device("cuda", ctx.device)
        self.seam = torch.empty(SEAM_BYTES, dtype=torch.uint8, device=dev)
        self.all = torch.empty(self.world * SEAM_BYTES, dtype=torch.uint8, device=dev)
        self.cap = shard_len // params.min + 4 + _lib.DSX_SEAM_MAX_CUTS
        self.out = torch.empty(self.cap, dtype=torch.int64, device=dev)
        self.n = ctypes.c_uint64()

    def run(self):
        import torch
        import torch.distributed as dist
        L, h = lib(), self.ctx.h
        check(L.dsx_shard_local(h, ctypes.c_void_p(self.d_ptr), self.halo, self.start, self.len,
                                self.total, ctypes.byref(self.params.c),
                                ctypes.c_void_p(self.seam.data_ptr()), DSX_SEAM_DEVICE), h)
        for _ in range(self.world + 1):
            if dist.get_backend(self.group) == "nccl":
                dist.all_gather_into_tensor(self.all, self.seam, group=self.group)
            else:  # e.g. gloo (CPU tensors only): stage through host memory
                mine = self.seam.cpu()
                bufs = [torch.empty_like(mine) for _ in range(self.world)]
                dist.all_gather(bufs, mine, group=self.group)
                self.all.copy_(torch.cat(bufs))
            torch.cuda.current_stream().synchronize()
            rc = L.dsx_shard_resolve(h, ctypes.c_void_p(self.all.data_ptr()), self.world,
                                     self.rank, ctypes.c_void_p(self.seam.data_ptr()),
                                     ctypes.c_void_p(self.out.data_ptr()), self.cap,
                                     ctypes.byref(self.n), DSX_SEAM_DEVICE | DSX_OUT_DEVICE)
            if rc != DSX_E_RESYNC:
                check(rc, h)
                return self.n.value
        raise RuntimeError("seam resolution did not settle within nranks rounds")

    def cuts(self):
        return self.out[:self.n.value].cpu().numpy().astype(np.uint64)


def shard_chunk(d_ptr, halo, shard_start, shard_len, total, params, ctx=None, group=None,
                device=None):
    """This rank's exact cut list (np.uint64 chunk end offsets c with
    shard_start < c <= shard_start + shard_len).  The seam records go through
    host memory and ``torch.distributed`` (any backend)."""
    import torch.distributed as dist
    ctx = ctx or _lib.default_context()
    L, h = lib(), ctx.h
    seam = _lib.Seam()
    check(L.dsx_shard_local(h, ctypes.c_void_p(d_ptr), halo, shard_start, shard_len, total,
                            ctypes.byref(params.c), ctypes.addressof(seam), 0), h)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cap = shard_len // params.min + 4 + _lib.DSX_SEAM_MAX_CUTS
    out = np.empty(cap, dtype=np.uint64)
    n = ctypes.c_uint64()
    for _ in range(world + 1):
        arr = seams_from_bytes(exchange_seams(seam_to_bytes(seam), group, device), world)
        rc = L.dsx_shard_resolve(h, ctypes.addressof(arr), world, rank, ctypes.addressof(seam),
                                 out.ctypes.data, cap, ctypes.byref(n), 0)
        if rc != DSX_E_RESYNC:
            check(rc, h)
            return out[:n.value].copy()
    raise RuntimeError("seam resolution did not settle within nranks rounds")
