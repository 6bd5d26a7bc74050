#!/usr/bin/env python3
"""Per-wave timeline of the line-aligned scan (DSX_SCAN_TRACE=1): start/end
spread over the wave slots, by wave index within the workgroup, for one
device-resident blob (uniform, default params)."""
import ctypes
import os
import sys

import numpy as np

os.environ["DSX_SCAN_TRACE"] = "1"
if os.environ.get("DSX_SCAN_VARIANT", "0") != "0":  # VARIANT 5: the diagnostic build
    os.environ.setdefault("DSX_LIB_PATH", os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "desync_amd", "libdsx_diag.so"))
print("scan_trace: importing torch", flush=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import desync_amd  # noqa: E402
from desync_amd import _lib  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
W = int(os.environ.get("DSX_SCANL_WAVES", "8"))
n = int(gib * (1 << 30))
ctx = _lib.Context(0)
L = _lib.lib()
t = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctx.h)
for i in range(3):
    print(f"scan_trace: call {i}", flush=True)
    desync_amd.cut_device(t.data_ptr(), n, 16384, 65536, 262144, ctx=ctx)
st = ctx.stats()
print(f"stats: chunks {st.chunks} candidates {st.candidates} repaired {st.repaired_segments} "
      f"dense {st.dense_fallbacks}")
ns, nw = ctypes.c_uint64(), ctypes.c_uint64()
_lib.check(L.dsx_debug_trace(ctx.h, None, 0, ctypes.byref(ns), ctypes.byref(nw)), ctx.h)
buf = np.zeros(3 * ns.value + 10 * nw.value, np.uint64)
_lib.check(L.dsx_debug_trace(ctx.h, buf.ctypes.data, buf.size, ctypes.byref(ns),
                             ctypes.byref(nw)), ctx.h)
tr = buf[:3 * ns.value].reshape(-1, 3).astype(np.int64)
wk = buf[3 * ns.value:].reshape(-1, 10).astype(np.int64)
tr = tr[tr[:, 1] > 0]
if os.environ.get("DSX_SCAN_VARIANT") == "5":
    # shader-clock cycles per wave and cycles spent waiting for the line DMA
    tot = (tr[:, 1] - tr[:, 0]).astype(np.float64)
    m = (1 << 21) - 1
    parts = {"vmcnt wait": tr[:, 2] & m, "line copy + lgkmcnt(0)": (tr[:, 2] >> 21) & m,
             "DMA issue": (tr[:, 2] >> 42) & m}
    q = [0, 10, 50, 90, 100]
    print(f"waves {len(tr)}  cycles per wave median {np.median(tot):.0f}")
    for k, v in parts.items():
        print(f"  {k:24s} fraction pct {q} {np.percentile(v / tot, q).round(4).tolist()}")
    sys.exit(0)
t0 = tr[:, 0].min()
st = (tr[:, 0] - t0) / 100.0  # us (100 MHz)
en = (tr[:, 1] - t0) / 100.0
print(f"waves {len(tr)}  regions/wave {np.bincount(tr[:, 2].astype(int)).tolist()}")
q = [0, 1, 10, 50, 90, 99, 100]
print("start us  pct", q, np.percentile(st, q).round(1).tolist())
print("end   us  pct", q, np.percentile(en, q).round(1).tolist())
wi = np.arange(len(tr)) % W
for w in range(W):
    print(f"  wave {w}: end median {np.median(en[wi == w]):7.1f}  max {en[wi == w].max():7.1f}")
wk = wk[wk[:, 4] > 0]
if len(wk):
    rel = (wk[:, :5] - t0) / 100.0
    cyc = (wk[:, 6] - wk[:, 5]) / np.maximum(1, wk[:, 3] - wk[:, 2]) * 100.0
    print(f"walk phase 1 shader clock MHz median {np.median(cyc):.0f}")
    print(f"walk workgroups {len(wk)} (times from the first scan wave start, us)")
    for i, name in enumerate(["entry", "counts", "staged", "walk1", "walk2"]):
        print(f"  {name:7s} pct {q} {np.percentile(rel[:, i], q).round(1).tolist()}")
    sub = (wk[:, 7:10] - t0) / 100.0
    for i, name in enumerate(["seek", "step1", "chain"]):
        print(f"  {name:7s} pct {q} {np.percentile(sub[:, i], q).round(1).tolist()}")
