#!/usr/bin/env python3
"""In-process A/B of IndexFromFile's one-window tail feeder (dsx_index.cpp,
TailFeeder): a 1 GiB page-cache file, `dsx_index_fd` under several feeder
settings and `dsx_cut_fd` (the same read without IDs), the cases alternating
call by call so that the box's drift in page-cache read speed falls on all of
them alike.  Needs the diagnostic build for DSX_FEED_THREADS:

  DSX_LIB_PATH=desync_amd/libdsx_diag.so python3 tools/feed_ab.py [--gib=N] [rounds] [case ...]

A case is name=THREADS:CUT[:READERS] (CUT -1 = the default, else
DSX_INDEX_HOST_TAIL; READERS = DSX_INDEX_READERS, default 4) or `cut[:READERS]`
(dsx_cut_fd); a name starting with `v` times dsx_ids_fd (VerifyIndex) of the
file's chunk list instead of dsx_index_fd.  Prints one JSON line: per case the median, min and max
GiB/s and the median ratio to dsx_cut_fd of the same round.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import desync_amd  # noqa: E402
from desync_amd import _lib  # noqa: E402

MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10


def main():
    args = sys.argv[1:]
    gib = 1
    if args and args[0].startswith("--gib="):
        gib = int(args.pop(0).split("=")[1])
    rounds = int(args[0]) if args else 8
    cases = args[1:] or ["t11=11:-1", "t8=8:-1", "t11c96=11:98304", "off=11:0", "cut"]
    n = gib << 30
    rng = np.random.default_rng(7)
    fd, path = tempfile.mkstemp(prefix="dsx_feed_")
    res = {c.split("=")[0]: [] for c in cases}
    ratio = {c.split("=")[0]: [] for c in cases}
    try:
        with os.fdopen(fd, "wb") as f:
            for _ in range(4 * gib):
                f.write(rng.integers(0, 256, 256 << 20, dtype=np.uint8).tobytes())
            # written back before timing: dirty pages flushed in the background
            # during the timed calls slow the reads (round 6, tools/window_dip.py)
            f.flush()
            os.fsync(f.fileno())
        # one context per cut (DSX_INDEX_HOST_TAIL is read when a context is
        # made; DSX_FEED_THREADS at each call): switching settings through the
        # pool would close and remake them
        def key(c):
            if c.startswith("cut"):
                f = c.split(":")
                return ("-1", f[1] if len(f) > 1 else "4")
            f = c.split("=")[1].split(":")
            return (f[1], f[2] if len(f) > 2 else "4")

        ctxs = {}
        for c in cases:
            k = key(c)
            if k not in ctxs:
                os.environ["DSX_INDEX_HOST_TAIL"], os.environ["DSX_INDEX_READERS"] = k
                ctxs[k] = _lib.Context(0)
        fdr = os.open(path, os.O_RDONLY)
        try:
            ends, _ = desync_amd.index_fd(fdr, MIN, AVG, MAX)
            for r in range(rounds + 1):  # (round 0 warms the contexts, not counted)
                times = {}
                # (the order rotates from round to round: no case always
                # follows the same one)
                for c in cases[r % len(cases):] + cases[:r % len(cases)]:
                    name = c.split("=")[0]
                    if os.environ.get("DSX_TAIL_LOG"):  # (the library's log lines follow)
                        print("case: %s" % name, file=sys.stderr, flush=True)
                    # (`_nomid` in the name: no GPU share of a one-window file
                    # during the read, DSX_FEED_MID=0 in the diagnostic build;
                    # `_mK`: the shares at the first K points 1/2, 3/4, 7/8, ...;
                    # `_eN`: the last segment's cut N KiB, DSX_FEED_CUT_END;
                    # `_nX`: the shares' cuts at X ns per byte, DSX_SHARE_NS;
                    # `_k0`: the shares on digest_kernel, DSX_SHARE_PC=0;
                    # `_tN`: the last N MiB in finer pieces, DSX_FINE_TAIL, 0 off;
                    # `_dN`: of slot / N bytes, DSX_FINE_DIV;
                    # `_sN`: the shares may end N us after the read, DSX_SHARE_SLACK;
                    # `_xN`: N hashers join once the reads are done, DSX_FEED_EXTRA;
                    # `_u0`: no shares in the last of several windows, DSX_SHARE_MULTI=0)
                    for v in ("DSX_FEED_MID", "DSX_FEED_CUT_END", "DSX_SHARE_NS", "DSX_SHARE_PC",
                              "DSX_FINE_TAIL", "DSX_FINE_DIV", "DSX_SHARE_SLACK", "DSX_FEED_EXTRA",
                              "DSX_SHARE_MULTI"):
                        os.environ.pop(v, None)
                    for part in name.split("_")[1:]:
                        if part == "nomid":
                            os.environ["DSX_FEED_MID"] = "0"
                        elif part[:1] == "m" and part[1:].isdigit():
                            pts, f = [], 0.5
                            for _ in range(int(part[1:])):
                                pts.append(repr(f))
                                f = 0.5 * (1 + f)
                            os.environ["DSX_FEED_MID"] = ",".join(pts) or "0"
                        elif part[:1] == "e" and part[1:].isdigit():
                            os.environ["DSX_FEED_CUT_END"] = str(int(part[1:]) << 10)
                        elif part[:1] == "n" and part[1:].isdigit():
                            os.environ["DSX_SHARE_NS"] = part[1:]
                        elif part[:1] == "t" and part[1:].isdigit():
                            os.environ["DSX_FINE_TAIL"] = str(int(part[1:]) << 20)
                        elif part[:1] == "d" and part[1:].isdigit():
                            os.environ["DSX_FINE_DIV"] = part[1:]
                        elif part[:1] == "s" and part[1:].isdigit():
                            os.environ["DSX_SHARE_SLACK"] = part[1:]
                        elif part[:1] == "k" and part[1:].isdigit():
                            os.environ["DSX_SHARE_PC"] = part[1:]
                        elif part[:1] == "x" and part[1:].isdigit():
                            os.environ["DSX_FEED_EXTRA"] = part[1:]
                        elif part[:1] == "u" and part[1:].isdigit():
                            os.environ["DSX_SHARE_MULTI"] = part[1:]
                    if c.startswith("cut"):
                        t0 = time.perf_counter()
                        desync_amd.cut_fd(fdr, MIN, AVG, MAX, ctx=ctxs[key(c)])
                    elif c.startswith("v"):  # VerifyIndex's IDs of the list (dsx_ids_fd)
                        os.environ["DSX_FEED_THREADS"] = c.split("=")[1].split(":")[0]
                        t0 = time.perf_counter()
                        desync_amd.ids_fd(fdr, 0, ends, ctx=ctxs[key(c)])
                    else:
                        os.environ["DSX_FEED_THREADS"] = c.split("=")[1].split(":")[0]
                        # (a name ending in `_nomulti`: no feeder on the last of several windows)
                        os.environ["DSX_FEED_MULTI"] = "0" if name.endswith("_nomulti") else "1"
                        t0 = time.perf_counter()
                        desync_amd.index_fd(fdr, MIN, AVG, MAX, ctx=ctxs[key(c)])
                    times[name] = time.perf_counter() - t0
                if r == 0:
                    continue
                for name, t in times.items():
                    res[name].append(n / t / (1 << 30))
                    if "cut" in times:  # (the case named `cut`: dsx_cut_fd, default readers)
                        ratio[name].append(times["cut"] / t)
        finally:
            os.close(fdr)
            for ctx in ctxs.values():
                ctx.close()
    finally:
        os.unlink(path)
    out = {}
    for name, v in res.items():
        out[name] = {"gibs_median": round(float(np.median(v)), 2), "gibs_min": round(min(v), 2),
                     "gibs_max": round(max(v), 2),
                     "ratio_to_cut_fd_median": round(float(np.median(ratio[name])), 3) if ratio[name] else None}
    print(json.dumps({"tool": "feed_ab", "gib": gib, "rounds": rounds, "cases": cases, "results": out}))


if __name__ == "__main__":
    main()
