#!/usr/bin/env python3
"""Paired A/B of library settings inside ONE process, on one 1 GiB blob.

The box's clock drifts by up to ~25 % over a few seconds of back-to-back
scans (profiles/r03/drift), so whole-run A/B comparisons are noise.  Here
every config gets its own library context (settings are read from the
environment when a context is created), and the calls alternate
A, B, C, A, B, C, ... so each config sees the same thermal history.

  python tools/ab_paired.py [--gib 1] [--rounds 30] CFG [CFG ...]
  CFG = 'NAME:VAR=VAL,VAR=VAL' (an empty list keeps the defaults)

Per config: mean / median / p10 / p90 of the HIP-event scan and stitch ms
of each call, and the median of the per-round ratio to the first config.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--workload", default="uniform", choices=["uniform", "dedup", "zeros"])
    ap.add_argument("--params", default="16384,65536,262144")
    ap.add_argument("cfgs", nargs="+")
    args = ap.parse_args()
    import torch
    from desync_amd import _lib
    import desync_amd

    L = _lib.lib()
    n = int(args.gib * (1 << 30))
    mn, avg, mx = (int(x) for x in args.params.split(","))
    names, ctxs = [], []
    base_env = dict(os.environ)
    for cfg in args.cfgs:
        name, _, kv = cfg.partition(":")
        os.environ.clear()
        os.environ.update(base_env)
        for item in filter(None, kv.split(",")):
            k, _, v = item.partition("=")
            os.environ[k] = v
        ctxs.append(_lib.Context(0))
        names.append(name)
    os.environ.clear()
    os.environ.update(base_env)
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    if args.workload == "uniform":
        _lib.check(L.dsx_gen_uniform(ctxs[0].h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), ctxs[0].h)
    elif args.workload == "dedup":
        _lib.check(L.dsx_gen_dedup(ctxs[0].h, ctypes.c_void_p(t.data_ptr()), 0, n, 2, 0.30),
                   ctxs[0].h)
    else:
        t.zero_()
    torch.cuda.synchronize()
    ref = None
    for c in ctxs:  # warm-up + agreement
        got = desync_amd.cut_device(t.data_ptr(), n, mn, avg, mx, ctx=c)
        if ref is None:
            ref = got
        assert np.array_equal(got, ref), "configs disagree on the cut list"
    scan = np.zeros((args.rounds, len(ctxs)))
    stitch = np.zeros_like(scan)
    for r in range(args.rounds):
        order = list(range(len(ctxs)))
        if r % 2:
            order.reverse()
        for i in order:
            desync_amd.cut_device(t.data_ptr(), n, mn, avg, mx, ctx=ctxs[i])
            st = ctxs[i].stats()
            scan[r, i] = st.scan_ms
            stitch[r, i] = st.stitch_ms
        if r % 10 == 9:
            print(f"ab_paired: round {r + 1}", file=sys.stderr, flush=True)
    out = {"gib": args.gib, "rounds": args.rounds, "workload": args.workload, "configs": {}}
    for i, name in enumerate(names):
        s = scan[:, i]
        out["configs"][name] = {
            "cfg": args.cfgs[i],
            "scan_ms_mean": round(float(s.mean()), 4),
            "scan_ms_median": round(float(np.median(s)), 4),
            "scan_ms_p10_p90": [round(float(np.percentile(s, 10)), 4),
                                round(float(np.percentile(s, 90)), 4)],
            "stitch_ms_median": round(float(np.median(stitch[:, i])), 4),
            "ratio_to_first_median": round(float(np.median(s / scan[:, 0])), 4),
        }
    print(json.dumps(out, indent=1))
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
