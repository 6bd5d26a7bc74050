#!/usr/bin/env python3
"""ChunkStream A/B inside one process (the box's noise cancels): runs of
ChunkStream over the same 512 MiB with settings alternated run by run.
  python3 tools/cs_ab.py [reps]
Settings as cases below (round 5 compared the clone copy split over two
threads with one -- 6.28 against 7.03 GiB/s median, not kept -- 1 vs 4
store workers, and the interpreter's GIL switch interval).  Prints one JSON line with each setting's median,
min and max GiB/s."""
import io
import json
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import desync_amd  # noqa: E402

MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10


class NullStore:
    def HasChunk(self, cid):
        return False

    def StoreChunk(self, chunk):
        pass


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = 512 << 20
    data = np.random.default_rng(5).integers(0, 256, n, dtype=np.uint8).tobytes()
    # (store workers, interpreter switch interval in s or None for the default)
    cases = {"w4": (4, None), "w1": (1, None), "w4_si100us": (4, 1e-4), "w1_si100us": (1, 1e-4)}
    res = {k: [] for k in cases}
    si0 = sys.getswitchinterval()
    for r in range(reps + 1):
        for name, (nw, si) in cases.items():
            sys.setswitchinterval(si or si0)
            t0 = time.perf_counter()
            idx = desync_amd.ChunkStream(None, desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX),
                                         NullStore(), nw)
            dt = time.perf_counter() - t0
            assert len(idx.Chunks) > 0
            sys.setswitchinterval(si0)
            if r:  # (the first round warms the context pool)
                res[name].append(n / dt / 2**30)
    print(json.dumps({k: {"median": round(statistics.median(v), 2), "min": round(min(v), 2),
                          "max": round(max(v), 2)} for k, v in res.items()}))


if __name__ == "__main__":
    main()
