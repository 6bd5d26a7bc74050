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

from .index import CaFormatExcludeNoDump, CaFormatSHA512256, FormatIndex, Index, IndexChunk


class Chunk:
    """chunk.go's Chunk, reduced to what a store needs: the ID and the
    uncompressed bytes."""

    def __init__(self, chunk_id: bytes, data: bytes):
        self._id = chunk_id
        self._data = data

    def ID(self) -> bytes:
        return self._id

    def Data(self) -> bytes:
        return self._data


class ChunkStorage:
    """chunkstorage.go: stores a chunk once per ID (an in-memory mark, undone
    if the store fails) and skips IDs the store already has.  Thread-safe."""

    def __init__(self, ws):
        self.ws = ws
        self._lock = threading.Lock()
        self._processed = set()

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
        with self._lock:
            self.chunks[chunk.ID()] = chunk.Data()


_BATCH = 64  # chunks per hand-off to the store workers
_READ_AHEAD = 256 << 20  # two of dsx_stream_ids' 128 MiB batches


def ChunkStream(ctx, c, ws, n):
    """index.go:138-234.  ``c`` is a desync_amd Chunker that has not produced
    a chunk yet (its IDs are switched on here), ``ws`` a store, ``n`` the
    number of store workers.  ``ctx``: an object with ``done()`` or None; when
    it reports done the producer stops and the chunks so far form the index,
    as the reference's select on ctx.Done() does (index.go:203-206).  A
    reader error (ChunkerReadError) or a store error is raised."""
    c.EnableIDs()
    if hasattr(c, "_ra"):
        # ChunkStream reads the stream to its end: the reader may run two ID
        # batches (2 x 128 MiB) ahead, so batches are scanned and hashed while
        # this thread hands out the chunks before them
        c._ra = max(c._ra, _READ_AHEAD)
    storage = ChunkStorage(ws)
    chunks = []
    nw = max(1, int(n))
    # the reference's channel to n store goroutines (index.go:150-182): a
    # bounded queue read by n threads; the first store error stops the
    # producer, the workers drain what is queued without storing it
    # (chunks travel in groups of up to _BATCH: a queue hand-off per chunk
    # cost more than the rest of the per-chunk work; each chunk is still
    # stored on its own, in stream order within a group)
    work = queue.Queue(maxsize=4 * nw)
    errors = []

    def worker():
        while True:
            group = work.get()
            if group is None:
                return
            for ch in group:
                if errors:
                    break
                try:
                    storage.StoreChunk(ch)
                except BaseException as e:  # noqa: BLE001 -- re-raised by the producer
                    errors.append(e)

    threads = [threading.Thread(target=worker, daemon=True) for _ in range(nw)]
    for t in threads:
        t.start()
    group = []
    done = getattr(ctx, "done", None) if ctx is not None else None
    run_of = getattr(c, "_next_run", None)  # (Next() for a run of chunks; this package's Chunker)
    try:
        while not errors:
            if run_of is not None:
                run = run_of()
            else:
                start, b = c.Next()
                run = [(start, bytes(b), c.ChunkID())] if b else []
            if not run:
                break
            stop = False
            for start, data, cid in run:  # data: a clone (slices.Clone, index.go:196-200)
                if done is not None and done():
                    stop = True
                    break
                if cid is None:
                    raise RuntimeError("chunker produced a chunk without a GPU chunk ID")
                chunks.append(IndexChunk(cid, start, len(data)))
                group.append(Chunk(cid, data))
                if len(group) >= _BATCH:
                    work.put(group)
                    group = []
            if stop:
                break
    finally:
        if group and not errors:
            work.put(group)
        for _ in threads:
            work.put(None)
        for t in threads:
            t.join()
    if errors:
        raise errors[0]
    return Index(FormatIndex(CaFormatExcludeNoDump | CaFormatSHA512256, c.Min(), c.Avg(), c.Max()),
                 chunks)
