"""ChopFile (chop.go:14-81): split a file by an index's chunk list and store
every chunk, checking each one against its ID on the way.

Reference shape: n workers, each with its own file handle, take index chunks
from a channel, read the chunk's bytes (readChunkFromFile, chop.go:66-81)
and build it with NewChunkWithID(id, b, skipVerify=false), which hashes the
bytes and fails with ChunkInvalid when they do not match the ID (chunk.go:37-73,
errors.go:23-43); valid chunks go to the store through a ChunkStorage.

Here the chunks are read in batches of contiguous chunks (up to 64 MiB): the
batch's bytes are read once, every chunk's Digest.Sum (SHA-512/256 or
SHA-256) is computed on the GPU from those bytes (dsx_ids_host), and the n
workers store exactly the bytes that were hashed -- the check and the store
see the same read, as NewChunkWithID's verify does (chop.go:76-80).  A
mismatching chunk is raised as ChunkInvalid when a worker reaches it, so the
chunks ahead of it may already be stored, as with the reference's workers; a
chunk past the end of the file raises EOFError (io.ReadFull's EOF /
ErrUnexpectedEOF).  Compression and the concrete stores stay out of scope (a
store is any object with HasChunk(id) and StoreChunk(chunk)).
"""
from __future__ import annotations

import os
import queue
import threading

import numpy as np

from .errors import ChunkInvalid
from .make import NullProgressBar, _chunk_runs, file_size, ids_host
from .stream import Chunk, ChunkStorage


_BATCH = 64 << 20  # bytes read (and hashed on the GPU) at once


def _batches(chunks, size):
    """(first index, chunks, bytes) per batch of contiguous chunks of at most
    _BATCH bytes (a longer chunk alone); the bytes are one read of the file,
    short at its end.  Chunks of a hand-built list need not be contiguous:
    each contiguous run is batched on its own."""
    i = 0
    for run in _chunk_runs(chunks):
        j = 0
        while j < len(run):
            k = j + 1
            while k < len(run) and run[k].Start + run[k].Size - run[j].Start <= _BATCH:
                k += 1
            yield i + j, run[j:k]
            j = k
        i += len(run)


def _read_hash(f, batch, size, device):
    """One read of the batch's bytes and the GPU IDs of the chunks inside
    them: (bytes, [id or None per chunk])."""
    start = batch[0].Start
    end = min(batch[-1].Start + batch[-1].Size, max(size, start))
    buf = os.pread(f.fileno(), end - start, start) if end > start else b""
    ends = np.fromiter((c.Start + c.Size - start for c in batch), dtype=np.uint64, count=len(batch))
    inside = int(np.searchsorted(ends, len(buf), side="right"))  # (ends non-decreasing)
    sums = [None] * len(batch)
    if inside:
        ids = ids_host(np.frombuffer(buf, np.uint8), 0, ends[:inside], device=device)
        for k in range(inside):
            sums[k] = ids[k].tobytes()
    return buf, sums


def ChopFile(ctx, name, chunks, ws, n, pb=None, device=0):
    """chop.go:14-64.  ``chunks``: IndexChunk list (e.g. ``Index.Chunks``),
    ``ws``: a WriteStore (HasChunk / StoreChunk), ``n``: worker count, ``ctx``:
    an object with ``done()`` or None (stops feeding the workers).  Raises the
    first worker error: ChunkInvalid, EOFError or the store's error."""
    pb = pb or NullProgressBar()
    pb.SetTotal(len(chunks))
    pb.Start()
    try:
        s = ChunkStorage(ws)
        files = []
        try:
            for _ in range(max(1, int(n))):
                try:
                    files.append(open(name, "rb"))
                except OSError as e:
                    raise OSError(f"unable to open file {name}, {e}") from e
            size = file_size(files[0].fileno())
            work = queue.Queue(maxsize=4 * len(files))
            errors = []
            stop = threading.Event()

            def worker():
                while True:
                    item = work.get()
                    if item is None:
                        return
                    if stop.is_set():
                        continue
                    c, b, got = item
                    try:
                        pb.Increment()
                        if got is None:  # (the chunk runs past the end of the file)
                            raise EOFError("EOF" if not b else "unexpected EOF")
                        if got != bytes(c.ID):
                            raise ChunkInvalid(c.ID, got)
                        s.StoreChunk(Chunk(bytes(c.ID), b))
                    except BaseException as e:  # noqa: BLE001 -- re-raised below
                        errors.append(e)
                        stop.set()

            threads = [threading.Thread(target=worker, daemon=True) for _ in files]
            for t in threads:
                t.start()
            try:
                for _, batch in _batches(chunks, size):
                    if stop.is_set() or (ctx is not None and getattr(ctx, "done", lambda: False)()):
                        break
                    buf, sums = _read_hash(files[0], batch, size, device)
                    base = batch[0].Start
                    for c, got in zip(batch, sums):
                        if stop.is_set():
                            break
                        lo = c.Start - base
                        work.put((c, buf[lo:lo + c.Size], got))
            finally:
                for _ in threads:
                    work.put(None)
                for t in threads:
                    t.join()
            if errors:
                raise errors[0]
        finally:
            for f in files:
                f.close()
    finally:
        pb.Finish()
    return None
