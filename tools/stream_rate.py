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
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ratestats import repeat  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = mib << 20
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    ctx = _lib.default_context(0)
    want = make.cut_host(np.frombuffer(data, np.uint8), MIN, AVG, MAX, ctx=ctx)
    def run_next(zero_copy):
        ch = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX, ctx=ctx, zero_copy=zero_copy)
        return [start + len(b) for start, b in ch]

    st_zc, ends = repeat(lambda: run_next(True), n)
    st_copy, ends_c = repeat(lambda: run_next(False), n)
    assert ends == ends_c
    assert np.array_equal(np.array(ends, dtype=np.uint64), want), "stream cut list differs"

    class NullStore:  # ChunkStream's store: keeps nothing (stores are out of scope)
        def HasChunk(self, cid):
            return False

        def StoreChunk(self, chunk):
            pass

    st_cs, idx = repeat(lambda: desync_amd.ChunkStream(
        None, desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX), NullStore(), 4), n)
    class PerChunk:  # the same Chunker without _next_run: ChunkStream's Next()-per-chunk path
        def __init__(self, c):
            object.__setattr__(self, "_c", c)

        def __getattr__(self, k):
            if k in ("_next_run", "_next_block"):
                raise AttributeError(k)
            return getattr(self._c, k)

        def __setattr__(self, k, v):
            setattr(self._c, k, v)

    st_pc, idx_pc = repeat(lambda: desync_amd.ChunkStream(
        None, PerChunk(desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)), NullStore(), 4), n)
    assert [(c.Start, c.Size, c.ID) for c in idx_pc.Chunks] == \
        [(c.Start, c.Size, c.ID) for c in idx.Chunks]
    got = np.array([c.Start + c.Size for c in idx.Chunks], dtype=np.uint64)
    assert np.array_equal(got, want), "ChunkStream cut list differs"
    import hashlib
    for c in (idx.Chunks[0], idx.Chunks[-1]):
        assert hashlib.new("sha512_256", data[c.Start:c.Start + c.Size]).digest() == c.ID
    print(json.dumps({"tool": "stream_rate", "mib": mib, "chunks": len(ends),
                      "gibs": st_zc["gibs_median"], "next_zero_copy": st_zc,
                      "next_copy_gibs": st_copy["gibs_median"], "next_copy": st_copy,
                      "chunkstream_gibs": st_cs["gibs_median"], "chunkstream": st_cs,
                      "chunkstream_per_chunk_gibs": st_pc["gibs_median"],
                      "chunkstream_per_chunk": st_pc,
                      "note": "io.BytesIO reader (readinto into the library's pinned buffer); "
                              "Next with zero_copy views (Go's aliasing rule) and with the "
                              "default bytes copy; ChunkStream = runs of chunks (Chunker._next_run) + GPU SHA-512/256 "
                              "IDs + bytes clone + store call per chunk; chunkstream_per_chunk = "
                              "the same through one Next() per chunk; medians of DSX_RATE_REPS "
                              "(10) runs with min/max"}))


if __name__ == "__main__":
    main()
