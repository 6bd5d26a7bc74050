"""Repaired segments of the bench workload (1 GiB uniform, seed 1): how often
the stitch takes fixup's sequential-repair path."""
import json
import sys

import torch

sys.path.insert(0, ".")
import desync_amd  # noqa: E402
from desync_amd import _lib  # noqa: E402

ctx = _lib.Context(0)
n = 1 << 30
t = torch.empty(n, dtype=torch.uint8, device="cuda")
import ctypes  # noqa: E402
L = _lib.lib()
_lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctx.h)
cuts = desync_amd.cut_device(t.data_ptr(), n, 16384, 65536, 262144, ctx=ctx)
print(json.dumps({"chunks": len(cuts), "repaired_segments": ctx.stats().repaired_segments}))
