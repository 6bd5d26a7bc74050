#!/usr/bin/env python3
"""Split-stream overlap: where and when does piece k's walk run beside piece
k+1's scan?  Queues 4 jobs on one context with DSX_SCAN_TRACE=2 (a trace slot
per piece) and prints, per piece, the scan's wave span and the walk's
workgroup entry / end times (s_memrealtime, 100 MHz) relative to the first
scan, and whether the walk's CUs were also scan CUs."""
import ctypes
import os
import sys

import numpy as np

os.environ["DSX_SCAN_TRACE"] = "2"
os.environ.setdefault("DSX_LIB_PATH", os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "desync_amd", "libdsx_diag.so"))  # traces: the diagnostic build
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from desync_amd import _lib  # noqa: E402
import desync_amd  # noqa: E402

n = 1 << 30
ctx = _lib.Context(0)
L = _lib.lib()
t = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctx.h)
p = desync_amd.Params(16384, 65536, 262144)
outs = [torch.empty(n // 16384 + 4, dtype=torch.int64, device="cuda") for _ in range(4)]
cnt = ctypes.c_uint64()
desync_amd.cut_device(t.data_ptr(), n, 16384, 65536, 262144, ctx=ctx)  # warm-up
for i in range(4):
    _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(t.data_ptr()), n, ctypes.byref(p.c),
                                ctypes.c_void_p(outs[i].data_ptr()), outs[i].numel(), ctypes.byref(cnt),
                                _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC), ctx.h)
for i in range(4):
    _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
ns, nw = ctypes.c_uint64(), ctypes.c_uint64()
_lib.check(L.dsx_debug_trace(ctx.h, None, 0, ctypes.byref(ns), ctypes.byref(nw)), ctx.h)
slot = 6 * ns.value + 10 * 65536
buf = np.zeros(4 * slot, np.uint64)
_lib.check(L.dsx_debug_trace(ctx.h, buf.ctypes.data, buf.size, ctypes.byref(ns), ctypes.byref(nw)), ctx.h)
t0 = None
recs = []
for k in range(4):
    b = buf[k * slot:(k + 1) * slot]
    sc = b[:6 * ns.value].reshape(-1, 6).astype(np.int64)
    sc = sc[sc[:, 1] > 0]
    wk = b[6 * ns.value:].reshape(-1, 10).astype(np.int64)
    wk = wk[wk[:, 0] > 0]
    if not len(sc):
        continue
    recs.append((k, sc, wk))
    t0 = sc[:, 3].min() if t0 is None else min(t0, sc[:, 3].min())
for k, sc, wk in sorted(recs, key=lambda r: r[1][:, 3].min()):
    scu = set(zip((sc[:, 2] >> 32) & 0xF, (sc[:, 2] >> 40) & 0xFF))
    print(f"slot {k}: scan entry {(sc[:, 3].min() - t0) / 100:8.1f} .. last end {(sc[:, 1].max() - t0) / 100:8.1f} us, "
          f"{len(scu)} CUs")
    if len(wk):
        wcu = set(zip((wk[:, 6] >> 32) & 0xF, (wk[:, 6] >> 8) & 0xFF))
        q = [0, 50, 100]
        print(f"   walk: {len(wk)} wgs entry pct {np.percentile((wk[:, 0] - t0) / 100, q).round(1).tolist()} "
              f"staged {np.percentile((wk[:, 2] - t0) / 100, q).round(1).tolist()} "
              f"done {np.percentile((wk[:, 4] - t0) / 100, q).round(1).tolist()}  CUs {len(wcu)}, "
              f"shared with any scan: {len(wcu & set().union(*[set(zip((r[1][:, 2] >> 32) & 0xF, (r[1][:, 2] >> 40) & 0xFF)) for r in recs]))}")
