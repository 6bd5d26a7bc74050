#!/usr/bin/env python3
"""The 1 / 2 / 4 GiB host-path rates side by side (round
5's make_rate.json read dsx_cut_fd 32.97 GiB/s at 2 GiB against 42.2 / 42.4 at
1 / 4 GiB).  One file per size, written and fsync'ed before any timing (so no
dirty-page writeback runs under a timed call), then dsx_cut_fd, dsx_index_fd
and dsx_ids_fd (VerifyIndex's re-hash) round-robin over sizes and calls, the
order rotating each round, so box drift falls on every point alike.  Then one
cold-cache pass per size: posix_fadvise(DONTNEED) drops the file's pages and
one dsx_index_fd reads it from the device (the host tail's second read of
the long chunks, ADVICE r05, is then a real second read unless the pages the
first read brought in stay cached).

Run on the GPU box: python tools/window_dip.py [rounds] [GiB ...]; prints one
JSON line.
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

MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10


def write(path, n, seed):
    rng = np.random.default_rng(seed)
    with open(path, "wb") as f:
        left = n
        while left:
            k = min(left, 256 << 20)
            f.write(rng.integers(0, 256, k, dtype=np.uint8).tobytes())
            left -= k
        f.flush()
        os.fsync(f.fileno())


def main():
    args = sys.argv[1:]
    rounds = int(args[0]) if args else 8
    sizes = [float(a) for a in args[1:]] or [1.0, 2.0, 4.0]
    tmp = os.environ.get("TMPDIR", tempfile.gettempdir())
    files, fds, lists = {}, {}, {}
    res = {}
    try:
        for g in sizes:
            p = os.path.join(tmp, f"dsx_dip_{g:g}")
            write(p, int(g * (1 << 30)), 11)
            files[g] = p
            fds[g] = os.open(p, os.O_RDONLY)
            lists[g] = desync_amd.cut_fd(fds[g], MIN, AVG, MAX)  # (warms the context too)
        calls = [(g, c) for g in sizes for c in ("cut_fd", "index_fd", "ids_fd")]
        for r in range(rounds + 1):
            order = calls[r % len(calls):] + calls[:r % len(calls)]
            for g, c in order:
                fd = fds[g]
                t0 = time.perf_counter()
                if c == "cut_fd":
                    desync_amd.cut_fd(fd, MIN, AVG, MAX)
                elif c == "index_fd":
                    desync_amd.index_fd(fd, MIN, AVG, MAX)
                else:
                    desync_amd.ids_fd(fd, 0, lists[g])
                dt = time.perf_counter() - t0
                if r:
                    res.setdefault(f"{c}@{g:g}", []).append(g / dt)
        out = {k: {"gibs_median": round(float(np.median(v)), 2), "gibs_min": round(min(v), 2),
                   "gibs_max": round(max(v), 2), "n": len(v)} for k, v in res.items()}
        cold = {}
        for g in sizes:
            for c in ("cut_fd", "index_fd"):
                os.posix_fadvise(fds[g], 0, 0, os.POSIX_FADV_DONTNEED)
                t0 = time.perf_counter()
                if c == "cut_fd":
                    desync_amd.cut_fd(fds[g], MIN, AVG, MAX)
                else:
                    desync_amd.index_fd(fds[g], MIN, AVG, MAX)
                cold[f"{c}@{g:g}"] = round(g / (time.perf_counter() - t0), 2)
        print(json.dumps({"tool": "window_dip", "rounds": rounds, "warm": out, "cold_gibs": cold,
                          "note": "files fsync'ed before timing; warm = page-cache reads, calls "
                                  "round-robin; cold = one call after POSIX_FADV_DONTNEED"}))
    finally:
        for fd in fds.values():
            os.close(fd)
        for p in files.values():
            os.unlink(p)


if __name__ == "__main__":
    main()
