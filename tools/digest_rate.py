#!/usr/bin/env python3
"""Chunk-ID rate: dsx_chunk_ids (SHA-512/256 and
SHA-256, one chunk per lane from a global queue) over a device-resident
uniform blob already cut at 16/64/256 KiB.  IDs land in host memory (32 B per
chunk, the call syncs).  A sample of IDs is checked with hashlib.

Prints one JSON line.  Run on the GPU box: python tools/digest_rate.py [GiB ...]
"""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from desync_amd import _lib, make  # noqa: E402

GiB = 1 << 30
MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ratestats import repeat  # noqa: E402


def main():
    sizes = [float(a) for a in sys.argv[1:]] or [1.0, 4.0]
    ctx = _lib.default_context(0)
    L = _lib.lib()
    rows = []
    for gib in sizes:
        n = int(gib * GiB)
        t = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        _lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctx.h)
        torch.cuda.synchronize()
        ends = make.cut_device(t.data_ptr(), n, MIN, AVG, MAX, ctx=ctx)
        row = {"gib": gib, "chunks": int(ends.size)}
        for name, algo in (("sha512-256", _lib.DSX_DIGEST_SHA512_256), ("sha256", _lib.DSX_DIGEST_SHA256)):
            st, ids = repeat(lambda: make.chunk_ids(t.data_ptr(), n, ends, 0, ctx=ctx, algo=algo), n)
            row[name + "_gibs"] = st["gibs_median"]
            row[name + "_ms"] = round(st["s_median"] * 1e3, 3)
            row[name] = st
            # the C call alone: IDs into a preallocated host array, no Python list
            e64 = np.ascontiguousarray(ends, dtype=np.uint64)
            raw = np.empty((e64.size, 32), dtype=np.uint8)
            sc, _ = repeat(lambda: _lib.check(L.dsx_chunk_ids(
                ctx.h, ctypes.c_void_p(t.data_ptr()), n, 0, e64.ctypes.data, e64.size,
                raw.ctypes.data, 0, algo), ctx.h), n)
            row[name + "_call_gibs"] = sc["gibs_median"]
            row[name + "_call"] = sc
            # spot-check a few IDs against hashlib
            starts = np.concatenate([[0], ends[:-1]])
            for i in (0, ends.size // 2, ends.size - 1):
                b = t[int(starts[i]):int(ends[i])].cpu().numpy().tobytes()
                want = hashlib.new("sha512_256", b).digest() if name == "sha512-256" \
                    else hashlib.sha256(b).digest()
                assert ids[i] == want, (name, i)
        rows.append(row)
        del t
        torch.cuda.empty_cache()
    print(json.dumps({"tool": "digest_rate", "params": "16/64/256 KiB", "rows": rows,
                      "note": "<algo>_gibs: make.chunk_ids wall time (the C call + the Python list of IDs); <algo>_call_gibs: dsx_chunk_ids alone incl. sync and 32 B/chunk D2H; blob resident"}))


if __name__ == "__main__":
    main()
