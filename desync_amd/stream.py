"""ChunkStream (index.go:138-234) over the GPU stream: a single-stream
Chunker feeds chunks to a store and the Index is built in chunk order.

Reference shape: the producer calls Next(), clones the bytes (the slice
aliases the chunker's buffer, index.go:196-200) and hands them to n workers
that compute the chunk ID (NewChunk -> Digest.Sum, index.go:165-169) and store
the chunk through a ChunkStorage (chunkstorage.go: stores each ID once, skips
IDs the store already has).  Here the chunk IDs come from the GPU, computed
next to the cuts (dsx_stream_ids), and the n workers only store.  The index
flags are the reference's: ExcludeNoDump | SHA512256 (index.go:224-230).
Compression and the concrete stores stay out of scope (a store is any object
with HasChunk(id) and StoreChunk(chunk)).
"""
from __future__ import annotations

import queue
import threading
import weakref

import numpy as np

from . import _lib
from .index import CaFormatExcludeNoDump, CaFormatSHA512256, ChunkArray, FormatIndex, Index


class Chunk:
    """chunk.go's Chunk, reduced to what a store needs: the ID and the
    uncompressed bytes.  ChunkStream's chunks hold a read-only view of the
    clone of their run's bytes (bytes(chunk.Data()) copies it out).  The
    store contract: the view is valid for as long as it is referenced, but it
    pins the whole pooled slab (8 MiB) or run behind it, so a store that
    keeps chunk bytes past StoreChunk copies them (MemoryStore does)."""

    __slots__ = ("_id", "_data")

    def __init__(self, chunk_id: bytes, data):
        self._id = chunk_id
        self._data = data

    def ID(self) -> bytes:
        return self._id

    def Data(self):
        return self._data


class ChunkStorage:
    """chunkstorage.go: stores a chunk once per ID (an in-memory mark, undone
    if the store fails) and skips IDs the store already has.  Thread-safe."""

    def __init__(self, ws):
        self.ws = ws
        self._lock = threading.Lock()
        self._processed = set()

    def _mark(self, ids):
        """Marks the IDs not processed yet (one lock for a hand-off of chunks)
        and returns their positions in ``ids``; a duplicate within ``ids``
        counts once, like consecutive StoreChunk calls."""
        proc, fresh = self._processed, []
        with self._lock:
            for i, cid in enumerate(ids):
                if cid not in proc:
                    proc.add(cid)
                    fresh.append(i)
        return fresh

    def _unmark(self, ids):
        with self._lock:
            for cid in ids:
                self._processed.discard(cid)

    def StoreChunk(self, chunk: Chunk):
        cid = chunk.ID()
        with self._lock:
            if cid in self._processed:
                return
            self._processed.add(cid)
        try:
            if self.ws.HasChunk(cid):
                return
            self.ws.StoreChunk(chunk)
        except BaseException:
            with self._lock:
                self._processed.discard(cid)
            raise


class MemoryStore:
    """A WriteStore in memory (test double; desync's stores are out of scope)."""

    def __init__(self):
        self.chunks = {}
        self._lock = threading.Lock()

    def HasChunk(self, cid: bytes) -> bool:
        with self._lock:
            return cid in self.chunks

    def StoreChunk(self, chunk: Chunk):
        # Chunk.Data() is a read-only view into ChunkStream's pooled slab (or
        # a whole run): a store that keeps the bytes takes its own copy, as
        # Go's Chunk owns its []byte, so one kept chunk does not pin the slab
        data = bytes(chunk.Data())
        with self._lock:
            self.chunks[chunk.ID()] = data


_BATCH = 64  # chunks per hand-off to the store workers
_READ_AHEAD = 256 << 20  # two of dsx_stream_ids' 128 MiB batches
_SLAB = 8 << 20  # bytes per clone slab (a run's clone; runs are cut to this size)
_COPY_THREADS = 4  # threads per clone (dsx_host_copy)


class _ClonePool:
    """Reused buffers for ChunkStream's clones of the chunk bytes.  A fresh
    multi-MiB bytes object per run is a fresh mapping: page faults and the
    kernel's zero fill on the producer, an unmap (TLB shootdowns) when a
    store worker drops the last chunk of it -- measured 3.5 GiB/s on the GPU
    box against 5.3 for per-chunk copies.  A slab goes back to the pool when
    every chunk view of it is gone (the store did not keep the bytes); while
    stores hold them, clones fall back to fresh copies."""

    def __init__(self, nslabs):
        self._free = []
        self._left = nslabs  # slabs not yet allocated
        self._lock = threading.Lock()

    def _release(self, slab):
        with self._lock:
            self._free.append(slab)

    def clone(self, src):
        n = len(src)
        slab = None
        if n <= _SLAB:
            with self._lock:
                if self._free:
                    slab = self._free.pop()
                elif self._left:
                    self._left -= 1
                    slab = np.empty(_SLAB, np.uint8)
        if slab is None:
            return memoryview(bytes(src))
        view = slab[:n]
        if n:  # (libdsx's copy pool, without the GIL: one memcpy thread was 16 ms of 65 per 512 MiB)
            _lib.check(_lib.lib().dsx_host_copy(view.ctypes.data, np.frombuffer(src, np.uint8).ctypes.data,
                                                n, _COPY_THREADS))
        # the chunks' memoryviews keep `view` alive; when the last goes, the
        # slab is free again
        weakref.finalize(view, self._release, slab)
        return memoryview(view).toreadonly()


def ChunkStream(ctx, c, ws, n):
    """index.go:138-234.  ``c`` is a desync_amd Chunker that has not produced
    a chunk yet (its IDs are switched on here), ``ws`` a store, ``n`` the
    number of store workers.  ``ctx``: an object with ``done()`` or None; when
    it reports done the producer stops and the chunks so far form the index,
    as the reference's select on ctx.Done() does (index.go:203-206).  A
    reader error (ChunkerReadError) or a store error is raised.

    The producer takes the chunks a run at a time as arrays
    (Chunker._next_block: ends, IDs, one clone of the run's bytes -- the
    reference's slices.Clone, index.go:196-200, done once per run), and the
    index is a ChunkArray over those arrays: no per-chunk Python object is
    made on the producer side.  The store workers build each Chunk (a view
    of its run's clone) as they store it."""
    c.EnableIDs()
    if hasattr(c, "_ra"):
        # ChunkStream reads the stream to its end: the reader may run two ID
        # batches (2 x 128 MiB) ahead, so batches are scanned and hashed while
        # this thread hands out the chunks before them
        c._ra = max(c._ra, _READ_AHEAD)
    storage = ChunkStorage(ws)
    nw = max(1, int(n))
    # the reference's channel to n store goroutines (index.go:150-182): a
    # bounded queue read by n threads; the first store error stops the
    # producer at its next hand-off (groups of up to _BATCH chunks), and the
    # workers drain what is queued without storing it
    work = queue.Queue(maxsize=nw)
    errors = []

    def worker():
        # ChunkStorage.StoreChunk per chunk, with the processed-ID marks taken
        # for the whole hand-off under one lock (the per-chunk lock was a
        # third of a worker's time); on a store error the chunk's mark and
        # those of the hand-off's unstored chunks are taken back
        has, store = ws.HasChunk, ws.StoreChunk
        while True:
            item = work.get()
            if item is None:
                return
            s, ends, idb, mv, base = item
            ids = [idb[j:j + 32] for j in range(0, len(idb), 32)]
            fresh = storage._mark(ids)
            for k, i in enumerate(fresh):
                if errors:
                    storage._unmark([ids[j] for j in fresh[k:]])
                    break
                cid = ids[i]
                try:
                    if not has(cid):
                        store(Chunk(cid, mv[(ends[i - 1] if i else s) - base:ends[i] - base]))
                except BaseException as ex:  # noqa: BLE001 -- re-raised by the producer
                    storage._unmark([ids[j] for j in fresh[k:]])
                    errors.append(ex)
                    break

    threads = [threading.Thread(target=worker, daemon=True) for _ in range(nw)]
    for t in threads:
        t.start()
    done = getattr(ctx, "done", None) if ctx is not None else None
    block_of = getattr(c, "_next_block", None)  # (this package's Chunker)
    pool = _ClonePool(nw + 4)  # (queued groups + the block in hand + slack)
    all_ends, all_ids, first = [], bytearray(), None
    try:
        while not errors:
            if block_of is not None:
                blk = block_of(pool.clone, _SLAB)
            else:  # any object with Next() / ChunkID()
                s0, b = c.Next()
                blk = (s0, [s0 + len(b)], c.ChunkID() or b"", bytes(b)) if b else None
            if blk is None:
                break
            s0, ends, idb, data = blk
            if len(idb) != 32 * len(ends):
                raise RuntimeError("chunker produced a chunk without a GPU chunk ID")
            if first is None:
                first = s0
            m, stop = len(ends), False
            if done is not None:  # the reference's per-chunk select on ctx.Done()
                for i in range(m):
                    if done():
                        m, stop = i, True
                        break
            mv = data if isinstance(data, memoryview) else memoryview(data)
            for g in range(0, m, _BATCH):
                if errors:
                    break
                h = min(m, g + _BATCH)
                work.put((s0 if g == 0 else ends[g - 1], ends[g:h], idb[32 * g:32 * h], mv, s0))
            all_ends.extend(ends[:m])
            all_ids += idb[:32 * m]
            if stop:
                break
    finally:
        for _ in threads:
            work.put(None)
        for t in threads:
            t.join()
    if errors:
        raise errors[0]
    return Index(FormatIndex(CaFormatExcludeNoDump | CaFormatSHA512256, c.Min(), c.Avg(), c.Max()),
                 ChunkArray(all_ends, bytes(all_ids), first or 0))
