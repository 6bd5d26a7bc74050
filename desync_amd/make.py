"""IndexFromFile and the one-shot cut-list entry points (make.go).

Reference interface (make.go):
    func IndexFromFile(ctx context.Context, name string, n int,
                       min, avg, max uint64, pb ProgressBar)
        (Index, ChunkingStats, error)                                  :22-27
    type ChunkingStats struct{ ChunksAccepted, ChunksProduced uint64 }   :330-333

The reference fans the Chunker out over n goroutines (split-and-align); here
the whole cut list comes from the GPU (dsx_cut_fd: pinned H2D pipeline ->
scan -> stitch), so ``n`` only caps the host threads hashing chunk IDs.
Chunk IDs (Digest.Sum, make.go:223) are computed on the host with the
reference's algorithm (SHA-512/256 by default) -- the GPU digest is the next
step.
"""
from __future__ import annotations

import ctypes
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass

import numpy as np

from . import _lib, digest
from ._lib import DSX_OUT_DEVICE, DSX_OUT_HOST, check, lib
from .chunker import Params
from .errors import Interrupted
from .index import CaFormatExcludeNoDump, CaFormatSHA512256, FormatIndex, Index, IndexChunk, \
    catar_feature_flags


@dataclass
class ChunkingStats:
    """make.go:329-341"""

    ChunksAccepted: int = 0
    ChunksProduced: int = 0


class NullProgressBar:
    """nullprogressbar.go: a ProgressBar that does nothing."""

    def SetTotal(self, total):
        pass

    def Start(self):
        pass

    def Set(self, current):
        pass

    def Finish(self):
        pass


def _ends_buffer(length, min_size):
    cap = length // min_size + 2
    return np.empty(cap, dtype=np.uint64), cap


def cut_host(data, min_size, avg_size, max_size, ctx=None):
    """Host-memory blob -> chunk end offsets (np.uint64), via dsx_cut_host."""
    p = Params(min_size, avg_size, max_size)
    ctx = ctx or _lib.default_context()
    mv = memoryview(data).cast("B") if not isinstance(data, np.ndarray) else data
    arr = np.frombuffer(mv, dtype=np.uint8) if not isinstance(mv, np.ndarray) else mv
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    out, cap = _ends_buffer(arr.size, min_size)
    n = ctypes.c_uint64()
    check(lib().dsx_cut_host(ctx.h, arr.ctypes.data, arr.size, ctypes.byref(p.c), out.ctypes.data,
                             cap, ctypes.byref(n)), ctx.h)
    return out[:n.value].copy()


def cut_fd(fd, min_size, avg_size, max_size, offset=0, length=None, ctx=None):
    """File range -> chunk end offsets relative to ``offset`` (dsx_cut_fd)."""
    p = Params(min_size, avg_size, max_size)
    ctx = ctx or _lib.default_context()
    if length is None:
        length = os.fstat(fd).st_size - offset
    out, cap = _ends_buffer(length, min_size)
    n = ctypes.c_uint64()
    check(lib().dsx_cut_fd(ctx.h, fd, offset, length, ctypes.byref(p.c), out.ctypes.data, cap,
                           ctypes.byref(n)), ctx.h)
    return out[:n.value].copy()


def cut_device(ptr, length, min_size, avg_size, max_size, ctx=None, out_ptr=None, out_cap=0,
               sync=True):
    """Device-resident blob (HBM pointer, e.g. ``tensor.data_ptr()``) -> cut list.

    With ``out_ptr`` (a device buffer of ``out_cap`` uint64) the cuts stay in
    HBM and the count is returned; otherwise a host np.uint64 array.  With
    ``sync=False`` (device output only) the call only enqueues; finish with
    :func:`cut_device_result`.
    """
    p = Params(min_size, avg_size, max_size)
    ctx = ctx or _lib.default_context()
    n = ctypes.c_uint64()
    if out_ptr is not None:
        flags = DSX_OUT_DEVICE | (0 if sync else _lib.DSX_NO_SYNC)
        check(lib().dsx_cut_device(ctx.h, ctypes.c_void_p(ptr), length, ctypes.byref(p.c),
                                   ctypes.c_void_p(out_ptr), out_cap, ctypes.byref(n), flags),
              ctx.h)
        return n.value
    out, cap = _ends_buffer(length, min_size)
    check(lib().dsx_cut_device(ctx.h, ctypes.c_void_p(ptr), length, ctypes.byref(p.c),
                               out.ctypes.data, cap, ctypes.byref(n), DSX_OUT_HOST), ctx.h)
    return out[:n.value].copy()


def cut_device_result(ctx=None):
    ctx = ctx or _lib.default_context()
    n = ctypes.c_uint64()
    check(lib().dsx_result(ctx.h, ctypes.byref(n)), ctx.h)
    return n.value


def IndexFromFile(ctx, name, n, min_size, avg_size, max_size, pb=None, device=0):
    """make.go:22-163 -- chunk a file into an Index (not stored anywhere).

    ``ctx`` mirrors the Go context: any object with a ``done()`` method (or
    None); when it reports done, Interrupted is raised (make.go:201-203).
    """
    pb = pb or NullProgressBar()
    stats = ChunkingStats()
    flags = CaFormatExcludeNoDump
    if digest.Digest.Algorithm() == "sha512-256":
        flags |= CaFormatSHA512256  # make.go:35-38
    params = Params(min_size, avg_size, max_size)  # NewChunker validation, make.go:103
    index = Index(FormatIndex(flags, min_size, avg_size, max_size), [])
    with open(name, "rb") as f:
        head = f.read(64)
        index.Index.FeatureFlags |= catar_feature_flags(head)  # make.go:49-61
        size = os.fstat(f.fileno()).st_size  # GetFileSize, make.go:64
        pb.SetTotal(size)
        pb.Start()
        try:
            if ctx is not None and getattr(ctx, "done", lambda: False)():
                raise Interrupted()
            dctx = _lib.default_context(device)
            ends = cut_fd(f.fileno(), min_size, avg_size, max_size, 0, size, ctx=dctx)
            starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64) if ends.size else ends
            ids = _chunk_ids(f.fileno(), starts, ends, max(1, int(n)))
            for s, e, cid in zip(starts.tolist(), ends.tolist(), ids):
                index.Chunks.append(IndexChunk(ID=cid, Start=s, Size=e - s))
                pb.Set(e)
            stats.ChunksAccepted = len(index.Chunks)
            stats.ChunksProduced = len(index.Chunks)
        finally:
            pb.Finish()
    del params
    return index, stats


def _chunk_ids(fd, starts, ends, n):
    """Digest.Sum per chunk (make.go:223); n host threads."""
    def one(i):
        s, e = int(starts[i]), int(ends[i])
        return digest.Digest.Sum(os.pread(fd, e - s, s))

    idx = range(len(starts))
    if n <= 1 or len(starts) < 2:
        return [one(i) for i in idx]
    with ThreadPoolExecutor(max_workers=n) as ex:
        return list(ex.map(one, idx))
