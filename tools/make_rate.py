#!/usr/bin/env python3
"""End-to-end `desync make` rate (IndexFromFile, make.go:22-163): a file in
the page cache -> HBM -> cut list -> chunk IDs (SHA-512/256) -> Index, plus
the caibx bytes (Index.WriteTo); then VerifyIndex of the same index
(verifyindex.go:13-79: the chunk list re-hashed through dsx_ids_fd).  The file is seeded uniform bytes written to
$TMPDIR; the cut list is checked against dsx_cut_host on the same bytes and
three chunk IDs with hashlib.

Prints one JSON line.  Run on the GPU box: python tools/make_rate.py [GiB ...]
"""
import hashlib
import io
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import desync_amd  # noqa: E402

MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ratestats import repeat  # noqa: E402


def main():
    sizes = [float(a) for a in sys.argv[1:]] or [1.0, 4.0]
    rows = []
    for gib in sizes:
        n = int(gib * (1 << 30))
        rng = np.random.default_rng(7)
        fd, path = tempfile.mkstemp(prefix="dsx_make_")
        try:
            with os.fdopen(fd, "wb") as f:
                left = n
                while left:
                    k = min(left, 256 << 20)
                    f.write(rng.integers(0, 256, k, dtype=np.uint8).tobytes())
                    left -= k
                f.flush()
                os.fsync(f.fileno())  # (no writeback during the timed calls)
            def make():
                index, stats = desync_amd.IndexFromFile(None, path, 1, MIN, AVG, MAX)
                b = io.BytesIO()
                index.WriteTo(b)
                return index, stats, b

            st_make, (index, stats, b) = repeat(make, n)
            fdr = os.open(path, os.O_RDONLY)
            try:
                st_idx, _ = repeat(lambda: desync_amd.index_fd(fdr, MIN, AVG, MAX), n)
                st_cut, _ = repeat(lambda: desync_amd.cut_fd(fdr, MIN, AVG, MAX), n)
            finally:
                os.close(fdr)
            # VerifyIndex over the index just made (dsx_ids_fd: file -> HBM -> IDs)
            st_ver, _ = repeat(lambda: desync_amd.VerifyIndex(None, path, index, 1), n)
            raw = np.fromfile(path, dtype=np.uint8)
            want = desync_amd.cut_host(raw, MIN, AVG, MAX)
            got = np.array([c.Start + c.Size for c in index.Chunks], dtype=np.uint64)
            assert np.array_equal(got, want), "cut list differs from dsx_cut_host"
            for c in (index.Chunks[0], index.Chunks[len(index.Chunks) // 2], index.Chunks[-1]):
                piece = raw[c.Start:c.Start + c.Size].tobytes()
                assert hashlib.new("sha512_256", piece).digest() == c.ID
            del raw
            rows.append({"gib": gib, "chunks": stats.ChunksAccepted, "caibx_bytes": len(b.getvalue()),
                         "gibs": st_make["gibs_median"], "index_fd_gibs": st_idx["gibs_median"],
                         "cut_fd_gibs": st_cut["gibs_median"], "verify_gibs": st_ver["gibs_median"],
                         "make": st_make, "index_fd": st_idx, "cut_fd": st_cut, "verify": st_ver})
        finally:
            os.unlink(path)
    print(json.dumps({"tool": "make_rate", "params": "16/64/256 KiB", "digest": "sha512-256",
                      "rows": rows, "note": "page-cache file -> HBM -> cuts + IDs -> caibx bytes (IndexFromFile); index_fd = the C call alone (dsx_index_fd); cut_fd = the cut list alone (dsx_cut_fd); verify = VerifyIndex of that index (dsx_ids_fd); medians of DSX_RATE_REPS (10) runs with min/max"}))


if __name__ == "__main__":
    main()
