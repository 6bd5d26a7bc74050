#!/usr/bin/env python3
"""Driver of tools/skipscan.hip (libskipscan.so): the reference's min-skip on
the GPU, measured beside the product scan at the bench's shape (VERDICT r05
item 2).

  python tools/skipscan.py [--gib 32] [--check-gib 2] [--configs G:SPAN_MIB,...]
                           [--secs 2] [--marks-dir DIR]

1. Exactness, per configuration, on --check-gib of the seed-3 uniform blob:
   the spans' chains stitched at their merge points (make.go:277-327's
   result) must equal libdsx.so's dsx_cut_device cut list.
2. Rate, per configuration, on --gib (32: the bench's per-GPU shard):
   launches back to back for --secs (the board reaches its power plateau),
   mean ms per launch; the same for the product (dsx_cut_device, 4 jobs
   queued like bench.py).  With --marks-dir each timed window's
   {t0, t1, bytes} goes to DIR/<name>.marks.json for tools/smu_summary.py
   (run the whole script under tools/smu_sample.py).

Counters per configuration: lines staged (x 128 B / bytes = staged per input
byte), windows, cuts, jumps (corrective DMAs), overrun chunks past span ends
(the merges), failed merges, idle lane-windows (lanes of groups with no span
left while others still run: the tail imbalance), and the waves' end spread.
Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10
GiB = 1 << 30
NSTAT = 8
STAT_NAMES = ("lines", "windows", "jumps", "overrun_chunks", "failed_merges", "cuts", "spans",
              "idle_lane_windows")


def stitch(cuts, ncut, merge, cap, length):
    """The true chain from the spans' chains: span k's cuts up to its merge
    point m_k (the first cut it shares with span k+1's chain), then span
    k+1's from after m_k."""
    out = []
    prev = None
    for k in range(ncut.size):
        lst = cuts[k * cap:k * cap + min(int(ncut[k]), cap)]
        if prev is not None:
            i = int(np.searchsorted(lst, prev))
            if i >= lst.size or lst[i] != prev:
                raise AssertionError(f"span {k}: merge point {prev} of span {k - 1} not in its chain")
            lst = lst[i + 1:]
        m = int(merge[k])
        if m == 0xFFFFFFFFFFFFFFFF:
            raise AssertionError(f"span {k}: no merge within the overrun cap")
        out.append(lst[lst <= m])
        if m >= length:
            break
        prev = m
    return np.concatenate(out) if out else np.zeros(0, np.uint64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=32.0)
    ap.add_argument("--check-gib", type=float, default=2.0)
    ap.add_argument("--configs", default="1:2,2:1,2:2,4:1,4:2")
    ap.add_argument("--secs", type=float, default=2.0)
    ap.add_argument("--marks-dir", default=None)
    args = ap.parse_args()
    import torch

    import subprocess

    import desync_amd
    from desync_amd import _lib
    so = os.path.join(REPO, "tools", "libskipscan.so")
    src = os.path.join(REPO, "tools", "skipscan.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                               "-shared", "-fPIC", src, "-o", so])
    sk = ctypes.CDLL(so)
    sk.skipscan_run.restype = ctypes.c_int
    L = _lib.lib()
    ctx = _lib.Context(0)
    p = desync_amd.Params(MIN, AVG, MAX)
    assert p.c.discriminator % 2 == 1 and p.c.qbias == 1, "skipscan handles odd d (qBias 1) only"
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    configs = [tuple(float(x) for x in c.split(":")) for c in args.configs.split(",")]

    def gen(n):
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        _lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 3), ctx.h)
        torch.cuda.synchronize()
        return t

    def run(t, n, G, span, iters):
        nspans = (n + span - 1) // span
        cap = span // MIN + 48
        cuts = torch.empty(nspans * cap, dtype=torch.int64, device="cuda")
        ncut = torch.zeros(nspans, dtype=torch.int32, device="cuda")
        merge = torch.empty(nspans, dtype=torch.int64, device="cuda")
        queue = torch.zeros(1, dtype=torch.int32, device="cuda")
        stats = torch.zeros(NSTAT, dtype=torch.int64, device="cuda")
        stamps = torch.zeros(ncu * 8 * 2, dtype=torch.int64, device="cuda")
        ms = ctypes.c_float()
        vp = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
        rc = sk.skipscan_run(vp(t), ctypes.c_uint64(n), ctypes.c_uint64(MIN), ctypes.c_uint64(MAX),
                             ctypes.c_uint32(p.c.inverse_odd), ctypes.c_uint32(p.c.qmax),
                             ctypes.c_uint64(span), ctypes.c_int(G), vp(cuts), vp(ncut), vp(merge),
                             vp(queue), vp(stats), vp(stamps), ctypes.c_uint32(cap),
                             ctypes.c_int(iters), ctypes.byref(ms))
        if rc:
            raise RuntimeError(f"skipscan_run: {rc}")
        st = stats.cpu().numpy()
        sm = stamps.cpu().numpy().reshape(-1, 2)
        sm = sm[sm[:, 1] > 0]
        spread = float((sm[:, 1].max() - np.median(sm[:, 1])) / 100.0) if sm.size else None  # us (100 MHz)
        return ms.value, dict(zip(STAT_NAMES, (int(x) for x in st))), spread, (cuts, ncut, merge, cap)

    res = {"tool": "skipscan", "params": "16/64/256 KiB", "check_gib": args.check_gib,
           "gib": args.gib, "configs": []}
    # ---- exactness ----
    nchk = int(args.check_gib * GiB)
    t = gen(nchk)
    ref = desync_amd.cut_device(t.data_ptr(), nchk, MIN, AVG, MAX, ctx=ctx)
    checks = {}
    for G, smib in configs:
        span = int(smib * (1 << 20))
        _, st, _, (cuts, ncut, merge, cap) = run(t, nchk, int(G), span, 1)
        got = stitch(cuts.cpu().numpy().astype(np.uint64), ncut.cpu().numpy(),
                     merge.cpu().numpy().astype(np.uint64), cap, nchk)
        ok = bool(np.array_equal(got, ref))
        checks[f"{int(G)}:{smib:g}"] = {"exact": ok, "cuts": int(got.size), "ref_cuts": int(ref.size),
                                        "failed_merges": st["failed_merges"]}
        if not ok:
            d = np.nonzero(got[:min(got.size, ref.size)] != ref[:min(got.size, ref.size)])[0]
            checks[f"{int(G)}:{smib:g}"]["first_diff"] = int(d[0]) if d.size else min(got.size, ref.size)
    res["check"] = checks
    del t
    torch.cuda.empty_cache()
    # ---- rate at the bench's shape ----
    n = int(args.gib * GiB)
    t = gen(n)

    def marks(name, t0, t1, nbytes):
        if args.marks_dir:
            os.makedirs(args.marks_dir, exist_ok=True)
            with open(os.path.join(args.marks_dir, name + ".marks.json"), "w") as f:
                json.dump({"t0": t0, "t1": t1, "bytes": nbytes}, f)

    # the product: dsx_cut_device jobs, 4 queued (bench.py's steady state)
    cap = n // MIN + 4
    outs = [torch.empty(cap, dtype=torch.int64, device="cuda") for _ in range(4)]
    cnt = ctypes.c_uint64()

    def product_jobs(k):
        q = 0
        for s in range(k):
            if q == 4:
                _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
                q -= 1
            _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(t.data_ptr()), n, ctypes.byref(p.c),
                                        ctypes.c_void_p(outs[s % 4].data_ptr()), cap, ctypes.byref(cnt),
                                        _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC), ctx.h)
            q += 1
        while q:
            _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
            q -= 1

    product_jobs(3)
    t0 = time.perf_counter()
    product_jobs(3)
    per = (time.perf_counter() - t0) / 3
    k = max(5, int(args.secs / per))
    w0 = time.time()
    t0 = time.perf_counter()
    product_jobs(k)
    dt = (time.perf_counter() - t0) / k
    marks("product", w0, time.time(), n * k)
    res["product"] = {"ms_per_job": round(dt * 1e3, 4), "gibs": round(n / dt / GiB, 1),
                      "frac_of_8tbs": round(n / dt / 8e12, 4), "jobs": k,
                      "note": "dsx_cut_device (scan + stitch of 4 x 8 GiB pieces), 4 queued; "
                              "wall clock per job"}
    for G, smib in configs:
        span = int(smib * (1 << 20))
        name = f"g{int(G)}_s{smib:g}"
        run(t, n, int(G), span, 2)  # warm
        ms1, _, _, _ = run(t, n, int(G), span, 1)
        iters = max(3, int(args.secs * 1e3 / max(ms1, 1e-3)))
        w0 = time.time()
        ms, st, spread, _ = run(t, n, int(G), span, iters)
        marks(name, w0, time.time(), n * iters)
        lanes_windows = st["windows"] * 64
        res["configs"].append({
            "name": name, "groups_per_wave": int(G), "lanes_per_chain": 64 // int(G),
            "span_mib": smib, "ms_per_launch": round(ms, 4), "gibs": round(n / (ms / 1e3) / GiB, 1),
            "frac_of_8tbs": round(n / (ms / 1e3) / 8e12, 4), "iters": iters,
            "staged_bytes_per_input_byte": round(st["lines"] * 128 / n, 4),
            "cuts": st["cuts"], "spans": st["spans"], "jumps": st["jumps"],
            "windows_per_wave": round(st["windows"] / (ncu * 8), 1),
            "overrun_chunks_per_span": round(st["overrun_chunks"] / max(1, st["spans"]), 3),
            "failed_merges": st["failed_merges"],
            "idle_lane_fraction": round(st["idle_lane_windows"] / max(1, lanes_windows), 4),
            "wave_end_spread_us": round(spread, 1) if spread is not None else None,
            "stats": st})
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
