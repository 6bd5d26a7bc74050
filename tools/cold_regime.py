#!/usr/bin/env python3
"""Per-launch scan duration and shader clock from an idle GPU, then again
after a 1 s idle gap (DPM vs first touch).

Runs bench.py's N = 1 job loop (dsx_cut_device jobs queued 4 deep on one
context, no event between them) on a blob generated on the device, with the
scan launches stamped from inside the kernel (dsx_stamps_begin/end):
duration = last wave end - first wave start (s_memrealtime, 100 MHz), clock =
sum of the waves' s_memtime cycles / their s_memrealtime ticks x 100 MHz.

usage: cold_regime.py [--gib G] [--seed S] [--jobs J] [--idle0 S] [--gap S]
prints a table (t_ms = launch start in milliseconds after the first launch of
the series) and writes JSON to --out.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

GiB = 1 << 30
MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024


def series(ctx, L, p, d_ptr, n, outs, cap, jobs, depth=4):
    from desync_amd import _lib
    ctx.stamps_begin(jobs * ((n + (8 * GiB) - 1) // (8 * GiB)) + 8)
    cnt = ctypes.c_uint64()
    pend = 0
    t0 = time.perf_counter()
    for s in range(jobs):
        if pend == depth:
            _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
            pend -= 1
        _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(d_ptr), n, ctypes.byref(p.c),
                                    ctypes.c_void_p(outs[s % depth].data_ptr()), cap,
                                    ctypes.byref(cnt), _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC), ctx.h)
        pend += 1
    while pend:
        _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
        pend -= 1
    wall = time.perf_counter() - t0
    st = ctx.stamps_end()
    base = st[0].t_first
    rows = [{"i": i, "t_ms": (s.t_first - base) / 1e5, "ms": s.ms, "mhz": round(s.mhz, 1),
             "busy": round(s.busy, 4),
             "gbs": s.bytes / (s.ms / 1e3) / 1e9 if s.ms else 0.0,
             "gap_ms": ((s.t_first - st[i - 1].t_last) / 1e5) if i else 0.0}
            for i, s in enumerate(st)]
    return {"jobs": jobs, "wall_s": wall, "gibs": jobs * n / wall / GiB, "chunks": cnt.value,
            "launches": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--jobs", type=int, default=60)
    ap.add_argument("--idle0", type=float, default=2.0, help="idle seconds before series A")
    ap.add_argument("--gap", type=float, default=1.0, help="idle seconds between series A and B")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    import desync_amd
    from desync_amd import _lib
    torch.cuda.set_device(0)
    ctx = _lib.Context(0)
    L = _lib.lib()
    n = int(a.gib * GiB)
    blob = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(blob.data_ptr()), 0, n, a.seed), ctx.h)
    cap = n // MIN + 4
    outs = [torch.empty(cap, dtype=torch.int64, device="cuda") for _ in range(4)]
    p = desync_amd.Params(MIN, AVG, MAX)
    # one untimed job: code objects loaded, scratch sized (not a warm-up of the clock)
    desync_amd.cut_device(blob.data_ptr(), n, MIN, AVG, MAX, ctx=ctx)
    torch.cuda.synchronize()
    time.sleep(a.idle0)
    A = series(ctx, L, p, blob.data_ptr(), n, outs, cap, a.jobs)
    time.sleep(a.gap)
    B = series(ctx, L, p, blob.data_ptr(), n, outs, cap, a.jobs)
    res = {"gib": a.gib, "seed": a.seed, "idle0_s": a.idle0, "gap_s": a.gap,
           "A_from_idle": A, "B_after_gap": B,
           "note": "per scan launch: ms = in-kernel duration (s_memrealtime), mhz = mean shader "
                   "clock of its waves (s_memtime / s_memrealtime), t_ms = launch start in ms "
                   "after the series' first launch, gap_ms = idle before it"}
    for name, S in (("A (from idle)", A), ("B (after gap)", B)):
        print(f"== {name}: {S['jobs']} jobs, {S['gibs']:.1f} GiB/s wall")
        print(f"{'i':>4} {'t_ms':>9} {'scan_ms':>8} {'MHz':>7} {'GB/s':>7} {'gap_ms':>7} {'busy':>6}")
        for r in S["launches"]:
            print(f"{r['i']:4d} {r['t_ms']:9.3f} {r['ms']:8.4f} {r['mhz']:7.1f} {r['gbs']:7.0f} "
                  f"{r['gap_ms']:7.4f} {r['busy']:6.3f}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
