#!/usr/bin/env python3
"""Host-resident chunking rate: bytes start and end in host
memory, so the rate includes the pinned H2D pipeline of libdsx.

  dsx_cut_host: a pageable numpy buffer -> cut list in host memory
  dsx_cut_fd:   a file in the page cache -> cut list in host memory

Prints one JSON line.  Run on the GPU box: python tools/host_rate.py [GiB]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import ctypes  # noqa: E402

import torch  # noqa: E402

from desync_amd import _lib, make  # noqa: E402

GiB = 1 << 30
MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ratestats import repeat  # noqa: E402


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    n = int(gib * GiB)
    ctx = _lib.default_context()
    t = torch.empty(n, dtype=torch.uint8, device="cuda")  # synthetic bytes, made on the GPU
    _lib.check(_lib.lib().dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctx.h)
    torch.cuda.synchronize()  # the generator ran on the library's stream
    data = t.cpu().numpy()
    del t
    st_host, ends_h = repeat(lambda: make.cut_host(data, MIN, AVG, MAX), n)
    # cuts + SHA-512/256 IDs from host memory (the host tail hashes the
    # caller's bytes in place)
    st_ihost, _ = repeat(lambda: make.index_host(data, MIN, AVG, MAX), n)
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), delete=False) as f:
        data.tofile(f)
        f.flush()
        os.fsync(f.fileno())  # (no write-back under the timed calls)
        path = f.name
    try:
        fd = os.open(path, os.O_RDONLY)
        try:
            st_fd, ends_f = repeat(lambda: make.cut_fd(fd, MIN, AVG, MAX), n)
        finally:
            os.close(fd)
    finally:
        os.unlink(path)
    assert np.array_equal(ends_h, ends_f)
    print(json.dumps({
        "bytes": n,
        "chunks": int(len(ends_h)),
        "cut_host_gibs": st_host["gibs_median"],
        "index_host_gibs": st_ihost["gibs_median"],
        "index_host": st_ihost,
        "cut_fd_gibs": st_fd["gibs_median"],
        "cut_host": st_host,
        "cut_fd": st_fd,
        "note": "host memory -> pinned H2D pipeline -> scan + stitch -> cut list in host memory",
    }))


if __name__ == "__main__":
    main()
