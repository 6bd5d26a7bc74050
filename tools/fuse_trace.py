"""Per-wave timeline of a fused scan (DSX_FUSE=1, stitch behind the scan): scan
wave ends, task waves, tasks per wave and time per task phase (DSX_SCAN_TRACE;
the trace of the last queued scan).  DESIGN.md 4.2."""
import ctypes, os, sys
import numpy as np
os.environ["DSX_SCAN_TRACE"] = "1"
os.environ.setdefault("DSX_LIB_PATH", os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "desync_amd", "libdsx_diag.so"))  # traces: the diagnostic build
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import desync_amd
from desync_amd import _lib
n = 1 << 30
ctx = _lib.Context(0)
L = _lib.lib()
t = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctx.h)
p = desync_amd.Params(16384, 65536, 262144)
outs = [torch.empty(n // 16384 + 4, dtype=torch.int64, device="cuda") for _ in range(4)]
cnt = ctypes.c_uint64()
nj = int(sys.argv[1]) if len(sys.argv) > 1 else 40
pend = 0
for s in range(nj):
    if pend == 4:
        _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h); pend -= 1
    _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(t.data_ptr()), n, ctypes.byref(p.c),
               ctypes.c_void_p(outs[s % 4].data_ptr()), n // 16384 + 4, ctypes.byref(cnt),
               _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC), ctx.h)
    pend += 1
# read the trace of the last scan before the flush
ns, nw = ctypes.c_uint64(), ctypes.c_uint64()
torch.cuda.synchronize()
_lib.check(L.dsx_debug_trace(ctx.h, None, 0, ctypes.byref(ns), ctypes.byref(nw)), ctx.h)
buf = np.zeros(6 * ns.value + 10 * nw.value, np.uint64)
_lib.check(L.dsx_debug_trace(ctx.h, buf.ctypes.data, buf.size, ctypes.byref(ns), ctypes.byref(nw)), ctx.h)
while pend:
    _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h); pend -= 1
N = ns.value
tr = buf[:6 * N].reshape(-1, 6).astype(np.int64)
tk = buf[6 * N:6 * N + 6 * N].reshape(-1, 6).astype(np.int64)
live = tr[:, 1] > 0
t0 = tr[live, 3].min()
us = lambda x: (x - t0) / 100.0
q = [0, 1, 10, 50, 90, 99, 100]
print("waves", N, "live", live.sum())
print("scan end us pct", q, np.percentile(us(tr[live, 1]), q).round(1).tolist())
has = tk[:, 2] > 0
print("task waves", has.sum(), "spare", (has & ~live).sum(), "live+tasks", (has & live).sum())
if has.any():
    print("task start us pct", q, np.percentile(us(tk[has, 0]), q).round(1).tolist())
    print("task end   us pct", q, np.percentile(us(tk[has, 1]), q).round(1).tolist())
    nrun = tk[has, 2] & 0xFFFF; nfin = tk[has, 2] >> 16
    print("tasks per wave", np.bincount(nrun).tolist(), "finish tasks total", int(nfin.sum()), "all", int(nrun.sum()))
    dur = (tk[has, 1] - tk[has, 0]) / 100.0 / np.maximum(nrun, 1)
    print("us per task pct", q, np.percentile(dur, q).round(1).tolist())
    sp = has & ~live
    if sp.any():
        print("spare task end pct", q, np.percentile(us(tk[sp, 1]), q).round(1).tolist())
end_all = np.maximum(tr[:, 1], tk[:, 1])
print("kernel last end us", us(end_all.max()).round(1))
print("scan start us pct", q, np.percentile(us(tr[live, 0]), q).round(1).tolist())
print("scan entry us pct", q, np.percentile(us(tr[live, 3]), q).round(1).tolist())
if has.any():
    nw_ = (tk[has, 2] & 0xFFFF) - (tk[has, 2] >> 16)
    nf_ = tk[has, 2] >> 16
    print("per walk task: staging us", round(tk[has, 3].sum() / 100.0 / max(1, nw_.sum()), 2),
          "walking us", round(tk[has, 4].sum() / 100.0 / max(1, nw_.sum()), 2),
          "per finish task us", round(tk[has, 5].sum() / 100.0 / max(1, nf_.sum()), 2))
