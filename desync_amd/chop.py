"""ChopFile (chop.go:14-81): split a file by an index's chunk list and store
every chunk, checking each one against its ID on the way.

Reference shape: n workers, each with its own file handle, take index chunks
from a channel, read the chunk's bytes (readChunkFromFile, chop.go:66-81)
and build it with NewChunkWithID(id, b, skipVerify=false), which hashes the
bytes and fails with ChunkInvalid when they do not match the ID (chunk.go:37-73,
errors.go:23-43); valid chunks go to the store through a ChunkStorage.

Here the check is done on the GPU first: one dsx_ids_fd call per contiguous
run of chunks streams the run's bytes into HBM and hashes every chunk there
(Digest.Sum: SHA-512/256 or SHA-256).  The n workers then only read and store.
A mismatching chunk is raised as ChunkInvalid when a worker reaches it, so the
chunks ahead of it may already be stored, as with the reference's workers;
a chunk past the end of the file raises EOFError (io.ReadFull's EOF /
ErrUnexpectedEOF).  Compression and the concrete stores stay out of scope (a
store is any object with HasChunk(id) and StoreChunk(chunk)).
"""
from __future__ import annotations

import os
import queue
import threading

import numpy as np

from .errors import ChunkInvalid
from .make import NullProgressBar, _contiguous_runs, file_size, ids_fd
from .stream import Chunk, ChunkStorage


def _chunk_sums(f, chunks, device):
    """GPU IDs of every chunk that lies inside the file (None for the others)."""
    size = file_size(f.fileno())
    sums = [None] * len(chunks)
    i = 0
    for run in _contiguous_runs(chunks):
        ends = np.fromiter((c.Start + c.Size for c in run), dtype=np.uint64, count=len(run))
        inside = int(np.searchsorted(ends, size, side="right"))  # (ends non-decreasing)
        if inside:
            ids = ids_fd(f.fileno(), run[0].Start, ends[:inside], 0, size, device=device)
            for k in range(inside):
                sums[i + k] = ids[k].tobytes()
        i += len(run)
    return sums


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
            sums = _chunk_sums(files[0], chunks, device)
            work = queue.Queue(maxsize=4 * len(files))
            errors = []
            stop = threading.Event()

            def worker(f):
                fd = f.fileno()
                while True:
                    item = work.get()
                    if item is None:
                        return
                    if stop.is_set():
                        continue
                    k, c = item
                    try:
                        pb.Increment()
                        b = os.pread(fd, c.Size, c.Start)
                        if len(b) < c.Size:
                            raise EOFError("EOF" if not b else "unexpected EOF")
                        if sums[k] != bytes(c.ID):
                            raise ChunkInvalid(c.ID, sums[k])
                        s.StoreChunk(Chunk(bytes(c.ID), b))
                    except BaseException as e:  # noqa: BLE001 -- re-raised below
                        errors.append(e)
                        stop.set()

            threads = [threading.Thread(target=worker, args=(f,), daemon=True) for f in files]
            for t in threads:
                t.start()
            try:
                for item in enumerate(chunks):
                    if stop.is_set() or (ctx is not None and getattr(ctx, "done", lambda: False)()):
                        break
                    work.put(item)
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
