#!/usr/bin/env python3
"""Streaming Chunker.Next rate: desync_amd.Chunker over
an in-memory reader (io.BytesIO) of seeded uniform bytes, default 16/64/256 KiB,
every chunk's bytes returned to Python as in the reference's Next
(chunker.go:206-277).  The whole path is host-resident: reader -> push (host
buffer, batched H2D) -> scan + stitch on the GPU -> pop.  Cut list checked
against dsx_cut_host on the same bytes.

Prints one JSON line.  Run on the GPU box: python tools/stream_rate.py [MiB]
"""
import io
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import desync_amd  # noqa: E402
from desync_amd import _lib, make  # noqa: E402

MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = mib << 20
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    ctx = _lib.default_context(0)
    want = make.cut_host(np.frombuffer(data, np.uint8), MIN, AVG, MAX, ctx=ctx)
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        ch = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX, ctx=ctx)
        ends = []
        for start, b in ch:
            ends.append(start + len(b))
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    assert np.array_equal(np.array(ends, dtype=np.uint64), want), "stream cut list differs"

    class NullStore:  # ChunkStream's store: keeps nothing (stores are out of scope)
        def HasChunk(self, cid):
            return False

        def StoreChunk(self, chunk):
            pass

    best_cs = None
    for _ in range(3):
        t0 = time.perf_counter()
        idx = desync_amd.ChunkStream(None, desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX),
                                     NullStore(), 4)
        dt = time.perf_counter() - t0
        best_cs = dt if best_cs is None else min(best_cs, dt)
    got = np.array([c.Start + c.Size for c in idx.Chunks], dtype=np.uint64)
    assert np.array_equal(got, want), "ChunkStream cut list differs"
    import hashlib
    for c in (idx.Chunks[0], idx.Chunks[-1]):
        assert hashlib.new("sha512_256", data[c.Start:c.Start + c.Size]).digest() == c.ID
    print(json.dumps({"tool": "stream_rate", "mib": mib, "chunks": len(ends),
                      "gibs": round(n / best / (1 << 30), 2), "s": round(best, 4),
                      "chunkstream_gibs": round(n / best_cs / (1 << 30), 2),
                      "chunkstream_s": round(best_cs, 4),
                      "note": "io.BytesIO reader (readinto into the library's pinned buffer), "
                              "a zero-copy chunk view per Next; ChunkStream = Next + GPU "
                              "SHA-512/256 IDs + bytes clone + store call per chunk"}))


if __name__ == "__main__":
    main()
