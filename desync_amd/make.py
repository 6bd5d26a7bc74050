"""IndexFromFile and the one-shot cut-list entry points (make.go).

Reference interface (make.go):
    func IndexFromFile(ctx context.Context, name string, n int,
                       min, avg, max uint64, pb ProgressBar)
        (Index, ChunkingStats, error)                                  :22-27
    type ChunkingStats struct{ ChunksAccepted, ChunksProduced uint64 }   :330-333

The reference fans the Chunker out over n goroutines (split-and-align); here
the file is read into HBM once and both the cut list (scan -> stitch) and
the chunk IDs (Digest.Sum, make.go:223: SHA-512/256 by default, SHA-256
alternative) are computed on the GPU.
"""
from __future__ import annotations

import ctypes
import os
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

    def Add(self, n):
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


def chunk_ids(ptr, length, ends, start=0, ctx=None, algo=None):
    """Digest.Sum of every chunk of a device-resident blob on the GPU
    (dsx_chunk_ids; digest.go:11-29, make.go:223).  ``ends`` is a host array of
    chunk end offsets, the first chunk starts at ``start``.  Returns a list of
    32-byte IDs.  ``algo`` defaults to the package-global Digest."""
    ctx = ctx or _lib.default_context()
    if algo is None:
        algo = (_lib.DSX_DIGEST_SHA512_256 if digest.Digest.Algorithm() == "sha512-256"
                else _lib.DSX_DIGEST_SHA256)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    out = np.empty((ends.size, 32), dtype=np.uint8)
    if ends.size:
        check(lib().dsx_chunk_ids(ctx.h, ctypes.c_void_p(ptr), length, start, ends.ctypes.data,
                                  ends.size, out.ctypes.data, 0, algo), ctx.h)
    return [bytes(r) for r in out]


_PIECE = 64 << 20   # bytes per pinned staging slot
_SLOTS = 4          # slots in flight (reads of one overlap the H2D of the others)
_staging = {}       # device -> list of pinned host tensors, reused across calls


def _file_to_device(f, size, device):
    """The whole file in HBM (288 GB per MI355X).  Pieces of 64 MiB are read
    with os.preadv by a small thread pool (the GIL is released) into a ring of
    pinned slots and copied to the device asynchronously on a side stream, so
    page-cache reads and the PCIe transfer overlap."""
    import concurrent.futures as cf

    import torch
    dev = torch.device(f"cuda:{device}")
    t = torch.empty(max(size, 1), dtype=torch.uint8, device=dev)
    if size == 0:
        return t
    slots = _staging.get(device)
    if slots is None:
        slots = [torch.empty(_PIECE, dtype=torch.uint8).pin_memory() for _ in range(_SLOTS)]
        _staging[device] = slots
    fd = f.fileno()
    stream = torch.cuda.Stream(device=dev)
    done = [None] * _SLOTS  # event of the last H2D out of each slot
    npieces = (size + _PIECE - 1) // _PIECE

    def read(k):
        off = k * _PIECE
        n = min(_PIECE, size - off)
        mv = memoryview(slots[k % _SLOTS].numpy())[:n]
        got = 0
        while got < n:
            r = os.preadv(fd, [mv[got:]], off + got)
            if r <= 0:
                raise OSError(f"short read at offset {off + got}")
            got += r
        return n

    with cf.ThreadPoolExecutor(max_workers=_SLOTS) as pool:
        futs = {}
        for k in range(min(_SLOTS, npieces)):
            futs[k] = pool.submit(read, k)
        for k in range(npieces):
            n = futs.pop(k).result()
            slot = k % _SLOTS
            with torch.cuda.stream(stream):
                t[k * _PIECE:k * _PIECE + n].copy_(slots[slot][:n], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
            done[slot] = ev
            nxt = k + _SLOTS
            if nxt < npieces:
                ev.synchronize()  # the slot is free once its copy has landed
                futs[nxt] = pool.submit(read, nxt)
    stream.synchronize()
    return t


def IndexFromFile(ctx, name, n, min_size, avg_size, max_size, pb=None, device=0):
    """make.go:22-163 -- chunk a file into an Index (not stored anywhere).

    The file is read into HBM once; the cut list (dsx_cut_device) and the
    chunk IDs (dsx_chunk_ids) are computed there.  ``n`` (the reference's
    worker count) has no effect on the result, as in the reference.  ``ctx``
    mirrors the Go context: any object with a ``done()`` method (or None);
    when it reports done, Interrupted is raised (make.go:201-203).
    """
    pb = pb or NullProgressBar()
    stats = ChunkingStats()
    flags = CaFormatExcludeNoDump
    if digest.Digest.Algorithm() == "sha512-256":
        flags |= CaFormatSHA512256  # make.go:35-38
    Params(min_size, avg_size, max_size)  # NewChunker validation, make.go:103
    index = Index(FormatIndex(flags, min_size, avg_size, max_size), [])
    with open(name, "rb") as f:
        head = f.read(64)
        index.Index.FeatureFlags |= catar_feature_flags(head)  # make.go:49-61
        size = os.fstat(f.fileno()).st_size  # GetFileSize, make.go:64
        f.seek(0)
        pb.SetTotal(size)
        pb.Start()
        try:
            if ctx is not None and getattr(ctx, "done", lambda: False)():
                raise Interrupted()
            dctx = _lib.default_context(device)
            blob = _file_to_device(f, size, device)
            ends = cut_device(blob.data_ptr(), size, min_size, avg_size, max_size, ctx=dctx)
            if ctx is not None and getattr(ctx, "done", lambda: False)():
                raise Interrupted()
            ids = chunk_ids(blob.data_ptr(), size, ends, 0, ctx=dctx)
            del blob
            starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64) if ends.size else ends
            for s, e, cid in zip(starts.tolist(), ends.tolist(), ids):
                index.Chunks.append(IndexChunk(ID=cid, Start=s, Size=e - s))
                pb.Set(e)
            stats.ChunksAccepted = len(index.Chunks)
            stats.ChunksProduced = len(index.Chunks)
        finally:
            pb.Finish()
    return index, stats


class VerifyError(Exception):
    """The plain ``fmt.Errorf`` errors VerifyIndex returns (verifyindex.go:27,
    fileseed.go:192)."""


def _contiguous_runs(chunks):
    """Split index chunks into runs whose chunks follow each other (a decoded
    caibx is one run; a hand-built Index may have gaps or overlaps)."""
    i = 0
    while i < len(chunks):
        j = i + 1
        while j < len(chunks) and chunks[j].Start == chunks[j - 1].Start + chunks[j - 1].Size:
            j += 1
        yield chunks[i:j]
        i = j


def VerifyIndex(ctx, name, idx, n=1, pb=None, device=0):
    """verifyindex.go:13-79 -- re-calculate the chunk IDs of a blob and compare
    them with ``idx``.  Raises VerifyError on the first mismatch, as
    fileSeedSegment.Validate does (fileseed.go:183-196).

    The reference reads every chunk with ReadAt over ``n`` worker file handles;
    here the file is read into HBM once and all IDs are computed by
    dsx_chunk_ids (one launch per contiguous run of chunks).  ``n`` has no
    effect on the result.  Block/char devices skip the size check
    (verifyindex.go:26, isDevice)."""
    import stat as _stat
    pb = pb or NullProgressBar()
    pb.SetTotal(len(idx.Chunks))
    pb.Start()
    try:
        st = os.stat(name)
        is_dev = _stat.S_ISBLK(st.st_mode) or _stat.S_ISCHR(st.st_mode)
        if not is_dev and st.st_size != idx.Length():
            raise VerifyError(f"index size ({idx.Length()}) does not match file size ({st.st_size})")
        if ctx is not None and getattr(ctx, "done", lambda: False)():
            return None  # the reference stops feeding workers and returns g.Wait()
        if not idx.Chunks:
            return None
        need = max(c.Start + c.Size for c in idx.Chunks)
        with open(name, "rb") as f:
            size = os.fstat(f.fileno()).st_size if not is_dev else need
            if need > size:
                # ReadAt past the end of the file: io.EOF (fileseed.go:187)
                raise EOFError("EOF")
            dctx = _lib.default_context(device)
            blob = _file_to_device(f, need, device)
        for run in _contiguous_runs(idx.Chunks):
            if ctx is not None and getattr(ctx, "done", lambda: False)():
                break
            start = run[0].Start
            ends = np.fromiter((c.Start + c.Size for c in run), dtype=np.uint64, count=len(run))
            ids = chunk_ids(blob.data_ptr(), need, ends, start, ctx=dctx)
            for c, got in zip(run, ids):
                if got != bytes(c.ID):
                    raise VerifyError(f"seed index for {name} doesn't match its data")
            pb.Add(len(run))
        del blob
    finally:
        pb.Finish()
    return None
