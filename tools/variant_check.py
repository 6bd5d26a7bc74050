"""Cut list of a diagnostic scan variant (DSX_LIB_PATH=libdsx_diag.so,
DSX_SCAN_VARIANT=v) against the oracle on seeded blobs: for variants that
must stay results-exact (7: 4-byte table entries)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import desync_amd
from desync_amd import _lib
from oracle import oracle as o
ctx = _lib.Context(0)
for seed, n in ((3, (64 << 20) + 12345), (4, 1 << 30)):
    arr = o.synth_uniform(seed, 0, n) if n < (1 << 30) else None
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    import ctypes
    _lib.check(_lib.lib().dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, seed), ctx.h)
    host = t.cpu().numpy()
    got = desync_amd.cut_device(t.data_ptr(), n, 16384, 65536, 262144, ctx=ctx)
    ref = o.chunk_parallel(host, 16384, 65536, 262144, 16)
    assert np.array_equal(got, ref), f"variant differs at n={n}"
    print("ok", n, got.size, flush=True)
