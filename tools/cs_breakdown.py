#!/usr/bin/env python3
"""Where ChunkStream's time goes: over the same 512 MiB as
tools/stream_rate.py, times Next alone, Next with GPU chunk IDs, the producer
loop of ChunkStream without store threads, and ChunkStream with 1 and 4
workers (each a new Chunker: its context from the pool) and on one explicit
context; then a cProfile of one ChunkStream run.  Prints one JSON line and the
profile's top entries to stderr.  Run on the GPU box."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import desync_amd  # noqa: E402
from desync_amd.index import IndexChunk  # noqa: E402
from desync_amd.stream import Chunk  # noqa: E402

MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10


class NullStore:
    def HasChunk(self, cid):
        return False

    def StoreChunk(self, chunk):
        pass


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = mib << 20
    data = np.random.default_rng(5).integers(0, 256, n, dtype=np.uint8).tobytes()

    def next_only(ids):
        ch = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        if ids:
            ch.EnableIDs()
        k = 0
        while True:
            s, b = ch.Next()
            if not b:
                break
            if ids:
                ch.ChunkID()
            k += 1
        ch.close()
        return k

    def producer_only():
        ch = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        ch.EnableIDs()
        out = []
        while True:
            s, b = ch.Next()
            if not b:
                break
            cid = ch.ChunkID()
            d = bytes(b)
            out.append(IndexChunk(cid, s, len(d)))
            Chunk(cid, d)
        ch.close()
        return len(out)

    def blocks_only():  # ChunkStream's producer side: blocks with IDs, no store threads
        from desync_amd.stream import _ClonePool, _SLAB
        ch = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        ch.EnableIDs()
        ch._ra = 256 << 20
        pool, k = _ClonePool(8), 0
        while True:
            blk = ch._next_block(pool.clone, _SLAB)
            if blk is None:
                break
            k += len(blk[1])
        ch.close()
        return k

    def blocks_nocopy():  # the same without the clone: views dropped at once (measures the copy)
        ch = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        ch.EnableIDs()
        ch._ra = 256 << 20
        k = 0
        while True:
            blk = ch._next_block(lambda v: v, 8 << 20)
            if blk is None:
                break
            k += len(blk[1])
        ch.close()
        return k

    def read_only():  # the reader alone: BytesIO.readinto in 8 MiB pieces
        r, buf, k = io.BytesIO(data), bytearray(8 << 20), 0
        while r.readinto(buf):
            k += 1
        return k

    from desync_amd import _lib
    shared = _lib.Context(0)

    def cs(nw, ctx=None):
        ch = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX, ctx=ctx)
        k = len(desync_amd.ChunkStream(None, ch, NullStore(), nw).Chunks)
        ch.close()
        return k

    res = {"tool": "cs_breakdown", "mib": mib}
    for name, fn in (("next", lambda: next_only(False)), ("next_ids", lambda: next_only(True)),
                     ("producer", producer_only), ("blocks", blocks_only), ("blocks_nocopy", blocks_nocopy),
                     ("read_only", read_only), ("chunkstream_1", lambda: cs(1)),
                     ("chunkstream_4", lambda: cs(4)),
                     ("cs4_shared", lambda: cs(4, shared))):
        fn()  # warm-up
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            k = fn()
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[2]
        res[name] = {"s_median": round(t, 5), "gibs": round(n / t / 2**30, 2), "chunks": k,
                     "us_per_chunk": round(t / k * 1e6, 2), "min_s": round(min(ts), 5)}
    print(json.dumps(res))
    pr = cProfile.Profile()
    pr.enable()
    cs(4)
    pr.disable()
    pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
