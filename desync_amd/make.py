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
import stat as _stat
from dataclasses import dataclass

import numpy as np

from . import _lib, digest
from ._lib import DSX_OUT_DEVICE, DSX_OUT_HOST, check, lib
from .chunker import Params
from .errors import Interrupted
from .index import CaFormatExcludeNoDump, CaFormatSHA512256, ChunkArray, FormatIndex, Index, IndexChunk, \
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

    def Increment(self):
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
        length = max(0, file_size(fd) - offset)
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
    # one bytes object per row without a per-row numpy slice (7x faster at 256k IDs)
    return out.view("V32").ravel().tolist()


def file_size(fd):
    """GetFileSize (ioctl_linux.go:63-84): st_size for regular files, the
    BLKGETSIZE64 ioctl for block devices (whose st_size is 0)."""
    st = os.fstat(fd)
    if _stat.S_ISBLK(st.st_mode):
        import fcntl
        import struct
        BLKGETSIZE64 = 0x80081272
        return struct.unpack("Q", fcntl.ioctl(fd, BLKGETSIZE64, b"\0" * 8))[0]
    return st.st_size


def _digest_code(algo=None):
    if algo is None:
        algo = digest.Digest.Algorithm()
    if algo in ("sha512-256", _lib.DSX_DIGEST_SHA512_256):
        return _lib.DSX_DIGEST_SHA512_256
    if algo in ("sha256", _lib.DSX_DIGEST_SHA256):
        return _lib.DSX_DIGEST_SHA256
    raise ValueError(f"unknown digest {algo!r}")


class _CancelWatch:
    """Polls a Go-style ctx (``done()``) during a long library call and turns
    it into dsx_cancel (make.go:201-203 -> Interrupted)."""

    def __init__(self, ctx, dctx):
        import threading
        self.ctx, self.dctx = ctx, dctx
        self.stop = threading.Event()
        self.t = None
        if ctx is not None and hasattr(ctx, "done"):
            self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(0.02):
            if self.ctx.done():
                lib().dsx_cancel(self.dctx.h)
                return

    def __enter__(self):
        if self.t:
            self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        if self.t:
            self.t.join()
        return False


def _run_polled(fn, dctx, progress):
    """Runs the library call ``fn`` and, with a ``progress`` callback, reports
    dsx_progress to it from THIS thread while the call runs on a worker thread
    (ctypes releases the GIL), as IndexFromFile's main goroutine calls
    pb.Set per assembled chunk (make.go:134-140)."""
    if progress is None:
        return fn()
    import threading
    res = {}

    def work():
        try:
            res["rc"] = fn()
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            res["exc"] = e

    t = threading.Thread(target=work, daemon=True)
    t.start()
    v, last = ctypes.c_uint64(), 0
    while True:
        t.join(0.0005)
        if lib().dsx_progress(dctx.h, ctypes.byref(v)) == 0 and v.value > last:
            last = v.value
            progress(last)
        if not t.is_alive():
            break
    if "exc" in res:
        raise res["exc"]
    return res["rc"]


def _partial_error(rc, dctx, **partial):
    """Interrupted (make.go:201-203) or the I/O error, carrying the confirmed
    prefix the library returned with it (make.go:133-162 returns the chunks
    assembled so far next to the error)."""
    if rc == _lib.DSX_E_INTERRUPTED:
        err = Interrupted()
    else:
        try:
            check(rc, dctx.h)
        except _lib.DsxError as e:
            err = e
    for k, v in partial.items():
        setattr(err, k, v)
    return err


def index_fd(fd, min_size, avg_size, max_size, offset=0, length=None, algo=None, ctx=None,
             device=0, cancel=None, progress=None, stats=None):
    """dsx_index_fd: a file range -> (chunk end offsets relative to ``offset``,
    uint8 array of 32-byte chunk IDs), both computed on the GPU.  ``length``
    None means to the end (files and block devices).  ``progress(bytes)`` is
    called with the end of the last confirmed chunk as the call advances.  On
    cancellation (Interrupted) or a read error (DsxError DSX_E_IO) the raised
    exception carries the confirmed prefix as ``.ends`` / ``.ids``.  ``stats``
    (a dict) receives the call's dsx_stats_t fields."""
    p = Params(min_size, avg_size, max_size)
    code = _digest_code(algo)
    size = length if length is not None else max(0, file_size(fd) - offset)
    cap = size // min_size + 2
    ends = np.empty(cap, dtype=np.uint64)
    ids = np.empty((cap, 32), dtype=np.uint8)
    n = ctypes.c_uint64()

    def call(c):
        with _CancelWatch(cancel, c):
            rc = _run_polled(lambda: lib().dsx_index_fd(
                c.h, fd, offset, size, ctypes.byref(p.c), code, ends.ctypes.data,
                ids.ctypes.data, cap, ctypes.byref(n)), c, progress)
        if rc in (_lib.DSX_E_INTERRUPTED, _lib.DSX_E_IO):
            raise _partial_error(rc, c, ends=ends[:n.value].copy(), ids=ids[:n.value].copy())
        check(rc, c.h)
        if stats is not None:
            st = c.stats()
            stats.update({k: getattr(st, k) for k, _ in st._fields_})

    if ctx is not None:
        call(ctx)
    else:
        with _lib.pooled_context(device) as c:
            call(c)
    return ends[:n.value].copy(), ids[:n.value].copy()


def index_host(data, min_size, avg_size, max_size, algo=None, ctx=None, device=0):
    """dsx_index_host: a host-memory blob -> (chunk ends, chunk IDs) on the GPU."""
    p = Params(min_size, avg_size, max_size)
    code = _digest_code(algo)
    arr = np.ascontiguousarray(np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
                               if not isinstance(data, np.ndarray) else data, dtype=np.uint8)
    cap = arr.size // min_size + 2
    ends = np.empty(cap, dtype=np.uint64)
    ids = np.empty((cap, 32), dtype=np.uint8)
    n = ctypes.c_uint64()
    with (_lib.pooled_context(device) if ctx is None else _nullctx(ctx)) as c:
        check(lib().dsx_index_host(c.h, arr.ctypes.data, arr.size, ctypes.byref(p.c), code,
                                   ends.ctypes.data, ids.ctypes.data, cap, ctypes.byref(n)), c.h)
    return ends[:n.value].copy(), ids[:n.value].copy()


def _ids_call(fn, start, ends, algo, ctx, device, cancel=None):
    code = _digest_code(algo)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    ids = np.empty((ends.size, 32), dtype=np.uint8)

    def call(c):
        with _CancelWatch(cancel, c):
            rc = fn(c, code, ends, ids)
        if rc == _lib.DSX_E_INTERRUPTED:
            raise Interrupted()
        check(rc, c.h)

    if ends.size:
        if ctx is not None:
            call(ctx)
        else:
            with _lib.pooled_context(device) as c:
                call(c)
    return ids


def ids_fd(fd, start, ends, offset=0, length=None, algo=None, ctx=None, device=0, cancel=None):
    """dsx_ids_fd: Digest.Sum of the chunks [start, ends[0]), [ends[0], ends[1]),
    ... of a file range (offsets relative to ``offset``), read through the
    pinned pipeline into HBM and hashed there.  Returns an (n, 32) uint8 array."""
    size = length if length is not None else 0xFFFFFFFFFFFFFFFF
    return _ids_call(lambda c, code, e, out: lib().dsx_ids_fd(
        c.h, fd, offset, size, start, e.ctypes.data, e.size, code, out.ctypes.data),
        start, ends, algo, ctx, device, cancel)


def ids_host(data, start, ends, algo=None, ctx=None, device=0):
    """dsx_ids_host: as ids_fd for a host-memory blob."""
    arr = np.ascontiguousarray(np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
                               if not isinstance(data, np.ndarray) else data, dtype=np.uint8)
    return _ids_call(lambda c, code, e, out: lib().dsx_ids_host(
        c.h, arr.ctypes.data, arr.size, start, e.ctypes.data, e.size, code, out.ctypes.data),
        start, ends, algo, ctx, device)


class _nullctx:
    def __init__(self, v):
        self.v = v

    def __enter__(self):
        return self.v

    def __exit__(self, *exc):
        return False


def IndexFromFile(ctx, name, n, min_size, avg_size, max_size, pb=None, device=0):
    """make.go:22-163 -- chunk a file into an Index (not stored anywhere).

    One library call (dsx_index_fd) does the data path: reader threads stream
    the file (or block device) through pinned memory into HBM, where the cut
    list (scan + stitch) and the chunk IDs (Digest.Sum, SHA-512/256 or SHA-256)
    are computed.  ``n`` (the reference's worker count) has no effect on the
    result, as in the reference.  ``ctx`` mirrors the Go context: any object
    with a ``done()`` method (or None); when it reports done the call stops
    between 32 MiB pieces and Interrupted is raised (make.go:201-203).
    ``pb.Set`` receives the end of the last confirmed chunk while the call
    runs (dsx_progress), from the calling thread.  The reference returns
    ``(index, stats, err)``; here an error is raised and carries the chunks
    assembled before it as ``err.index`` / ``err.stats`` (the confirmed
    prefix of the chain, with IDs).
    """
    pb = pb or NullProgressBar()
    stats = ChunkingStats()
    flags = CaFormatExcludeNoDump
    if digest.Digest.Algorithm() == "sha512-256":
        flags |= CaFormatSHA512256  # make.go:35-38
    Params(min_size, avg_size, max_size)  # NewChunker validation, make.go:103
    index = Index(FormatIndex(flags, min_size, avg_size, max_size), [])

    call_stats = {}

    def assemble(ends, ids):
        index.Chunks = ChunkArray(ends, ids)  # (IndexChunk objects built on access)
        stats.ChunksAccepted = len(index.Chunks)
        # make.go:329-341 also counts the chunks workers produced and syncWith
        # dropped; here: the staged cuts a stitch repair replaced
        stats.ChunksProduced = len(index.Chunks) + int(call_stats.get("chunks_discarded", 0))

    with open(name, "rb") as f:
        head = f.read(64)
        index.Index.FeatureFlags |= catar_feature_flags(head)  # make.go:49-61
        size = file_size(f.fileno())  # GetFileSize, make.go:64
        pb.SetTotal(size)
        pb.Start()
        try:
            if ctx is not None and getattr(ctx, "done", lambda: False)():
                e = Interrupted()
                e.index, e.stats = index, stats
                raise e
            try:
                # pb.Set(chunk.Start + chunk.Size) as chunks are confirmed (make.go:138)
                ends, ids = index_fd(f.fileno(), min_size, avg_size, max_size, 0, size,
                                     device=device, cancel=ctx,
                                     progress=None if isinstance(pb, NullProgressBar) else pb.Set,
                                     stats=call_stats)
            except (Interrupted, _lib.DsxError) as e:
                # make.go:133-162 returns the chunks assembled so far with the
                # error: here the raised error carries them (.index, .stats)
                if getattr(e, "ends", None) is not None:
                    assemble(e.ends, e.ids)
                    if len(e.ends):
                        pb.Set(int(e.ends[-1]))
                e.index, e.stats = index, stats
                raise
            assemble(ends, ids)
            pb.Set(size)
        finally:
            pb.Finish()
    return index, stats


class VerifyError(Exception):
    """The plain ``fmt.Errorf`` errors VerifyIndex returns (verifyindex.go:27,
    fileseed.go:192)."""


def _chunk_arrays(chunks):
    """(starts, ends, ids (n, 32) uint8, bad) of an Index's chunks as arrays.
    A ChunkArray (IndexFromFile's result, a decoded caibx) already holds them:
    no IndexChunk is built.  ``bad`` marks chunks whose ID is not 32 bytes (a
    hand-built Index; a ChunkID is [32]byte in the reference, so they can only
    mismatch)."""
    if isinstance(chunks, ChunkArray) and chunks._list is None:
        ends = chunks._ends
        starts = np.empty_like(ends)
        if ends.size:
            starts[0] = 0
            starts[1:] = ends[:-1]
        return starts, ends, chunks._ids, None
    n = len(chunks)
    starts = np.fromiter((c.Start for c in chunks), dtype=np.uint64, count=n)
    ends = starts + np.fromiter((c.Size for c in chunks), dtype=np.uint64, count=n)
    raw = [bytes(c.ID) for c in chunks]
    bad = np.fromiter((len(r) != 32 for r in raw), dtype=bool, count=n)
    ids = np.frombuffer(b"".join(r if len(r) == 32 else bytes(32) for r in raw),
                        dtype=np.uint8).reshape(n, 32)
    return starts, ends, ids, (bad if bad.any() else None)


def _chunk_runs(chunks):
    """Runs of index chunks that follow each other, as lists of chunks
    (ChopFile batches each run on its own)."""
    i = 0
    while i < len(chunks):
        j = i + 1
        while j < len(chunks) and chunks[j].Start == chunks[j - 1].Start + chunks[j - 1].Size:
            j += 1
        yield chunks[i:j]
        i = j


def _contiguous_runs(starts, ends):
    """[lo, hi) index ranges of runs of chunks that follow each other (a
    decoded caibx is one run; a hand-built Index may have gaps or overlaps)."""
    cuts = (np.nonzero(starts[1:] != ends[:-1])[0] + 1).tolist()
    bounds = [0] + cuts + [int(starts.size)]
    return list(zip(bounds[:-1], bounds[1:]))


def VerifyIndex(ctx, name, idx, n=1, pb=None, device=0):
    """verifyindex.go:13-79 -- re-calculate the chunk IDs of a blob and compare
    them with ``idx``.  Raises VerifyError on the first mismatch, as
    fileSeedSegment.Validate does (fileseed.go:183-196).

    The reference reads every chunk with ReadAt over ``n`` worker file handles;
    here one library call per contiguous run of chunks (dsx_ids_fd) streams
    the run's bytes through pinned memory into HBM and hashes every chunk
    there.  ``n`` has no effect on the result.  Block/char devices skip the
    size check (verifyindex.go:26, isDevice)."""
    pb = pb or NullProgressBar()
    pb.SetTotal(len(idx.Chunks))
    pb.Start()
    try:
        st = os.stat(name)
        is_dev = _stat.S_ISBLK(st.st_mode) or _stat.S_ISCHR(st.st_mode)
        if not is_dev and st.st_size != idx.Length():
            raise VerifyError(f"index size ({idx.Length()}) does not match file size ({st.st_size})")
        if not idx.Chunks:
            return None
        starts, ends, want, bad = _chunk_arrays(idx.Chunks)
        with open(name, "rb") as f:
            size = file_size(f.fileno())
            if _stat.S_ISCHR(st.st_mode):  # (no size: read what the index covers)
                size = int(ends.max())
            for lo, hi in _contiguous_runs(starts, ends):
                if ctx is not None and getattr(ctx, "done", lambda: False)():
                    break  # the reference stops feeding workers and returns g.Wait()
                if int(ends[lo:hi].max()) > size:
                    # ReadAt past the end of the file: io.EOF (fileseed.go:187)
                    raise EOFError("EOF")
                got = ids_fd(f.fileno(), int(starts[lo]), ends[lo:hi], 0, size, device=device)
                differ = (got != want[lo:hi]).any(axis=1)
                if bad is not None:
                    differ |= bad[lo:hi]
                if differ.any():
                    raise VerifyError(f"seed index for {name} doesn't match its data")
                pb.Add(hi - lo)
    finally:
        pb.Finish()
    return None
