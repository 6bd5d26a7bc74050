#!/usr/bin/env python3
"""Per-wave timeline of the line-aligned scan (DSX_SCAN_TRACE=1): start/end
spread over the wave slots, by wave index within the workgroup, for one
device-resident blob (uniform, default params)."""
import ctypes
import os
import sys

import numpy as np

os.environ["DSX_SCAN_TRACE"] = "1"
os.environ.setdefault("DSX_LIB_PATH", os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "desync_amd", "libdsx_diag.so"))  # traces: the diagnostic build
print("scan_trace: importing torch", flush=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import desync_amd  # noqa: E402
from desync_amd import _lib  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
avg = int(sys.argv[2]) << 10 if len(sys.argv) > 2 else 65536  # (KiB; min = avg/4, max = 4 avg)
W = int(os.environ.get("DSX_SCANL_WAVES", "8"))
n = int(gib * (1 << 30))
ctx = _lib.Context(0)
L = _lib.lib()
t = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctx.h)
for i in range(3):
    print(f"scan_trace: call {i}", flush=True)
    desync_amd.cut_device(t.data_ptr(), n, avg // 4, avg, avg * 4, ctx=ctx)
st = ctx.stats()
st_scan_ms, st_stitch_ms = st.scan_ms, st.stitch_ms
print(f"stats: chunks {st.chunks} candidates {st.candidates} repaired {st.repaired_segments} "
      f"dense {st.dense_fallbacks}")
ns, nw = ctypes.c_uint64(), ctypes.c_uint64()
_lib.check(L.dsx_debug_trace(ctx.h, None, 0, ctypes.byref(ns), ctypes.byref(nw)), ctx.h)
buf = np.zeros(6 * ns.value + 10 * nw.value, np.uint64)
_lib.check(L.dsx_debug_trace(ctx.h, buf.ctypes.data, buf.size, ctypes.byref(ns),
                             ctypes.byref(nw)), ctx.h)
tr = buf[:6 * ns.value].reshape(-1, 6).astype(np.int64)
wk = buf[6 * ns.value:].reshape(-1, 10).astype(np.int64)
gid = np.arange(len(tr))[tr[:, 1] > 0]  # blockIdx * W + wave of the live waves
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
ent = (tr[:, 3] - t0) / 100.0
xcc = (tr[:, 2] >> 32) & 0xF
nreg = tr[:, 2] & 0xFFFFFFFF
print(f"waves {len(tr)}  regions/wave {np.bincount(nreg.astype(int)).tolist()}")
q = [0, 1, 10, 50, 90, 99, 100]
print(f"HIP-event scan ms of the traced call {st_scan_ms:.4f}, stitch ms {st_stitch_ms:.4f}; "
      f"first wave entry -> last wave end {en.max() - ent.min():.1f} us")
print("entry us  pct", q, np.percentile(ent, q).round(1).tolist())
multi = nreg > 1
if multi.any():  # region transitions: shader-clock cycles per transition
    per = (nreg[multi] - 1).astype(np.float64)
    print("per region transition, kcycles: region end -> next region pct [10, 50, 90]",
          np.percentile(tr[multi, 4] / per / 1e3, [10, 50, 90]).round(2).tolist(),
          " first-fetch waits", np.percentile(tr[multi, 5] / per / 1e3, [10, 50, 90]).round(2).tolist())
print("prologue (entry -> hashing start) us pct", q, np.percentile(st - ent, q).round(1).tolist())
print("start us  pct", q, np.percentile(st, q).round(1).tolist())
print("end   us  pct", q, np.percentile(en, q).round(1).tolist())
wi = gid % W
for w in range(W):
    print(f"  wave {w}: end median {np.median(en[wi == w]):7.1f}  max {en[wi == w].max():7.1f}")
full = nreg == np.bincount(nreg.astype(int)).argmax()  # waves with the common region count
for x in range(8):
    m = full & (xcc == x)
    if m.any():
        print(f"  xcc {x}: waves {m.sum():4d} end pct [10, 50, 90] "
              f"{np.percentile(en[m], [10, 50, 90]).round(1).tolist()}")
wg = gid // W
wg_end = np.array([en[(wg == g) & full].mean() if ((wg == g) & full).any() else np.nan
                   for g in range(wg.max() + 1)])
print("per-workgroup mean end us pct", q, np.nanpercentile(wg_end, q).round(1).tolist())
wsd = np.array([en[(wg == g) & full].std() for g in range(wg.max() + 1) if ((wg == g) & full).sum() > 1])
print("within-workgroup end std us pct", [10, 50, 90], np.percentile(wsd, [10, 50, 90]).round(2).tolist())
wk = wk[wk[:, 4] > 0]
if len(wk):
    rel = (wk[:, :5] - t0) / 100.0
    print(f"walk workgroups {len(wk)} (times from the first scan wave start, us)")
    for i, name in enumerate(["entry", "counts", "staged", "walk1", "walk2"]):
        print(f"  {name:7s} pct {q} {np.percentile(rel[:, i], q).round(1).tolist()}")
    for c, name in ((7, "seek"), (9, "chain")):
        print(f"  {name:7s} pct {q} {np.percentile((wk[:, c] - t0) / 100.0, q).round(1).tolist()}")
    print("walk phase durations per workgroup, us")
    for (i, j), name in (((0, 1), "counts"), ((1, 2), "staging"), ((2, 3), "phase 1"), ((3, 4), "phase 2"),
                         ((7, 9), "1st chain")):
        print(f"  {name:9s} pct {q} {np.percentile((wk[:, j] - wk[:, i]) / 100.0, q).round(2).tolist()}")
