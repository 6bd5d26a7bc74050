#!/usr/bin/env python3
"""One dsx_index_fd call over a page-cache file, for a kernel trace: run as
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/index_trace.py GIB
(GIB [--verify]: then two VerifyIndex calls of the list); then
tools/index_trace.py --summary DIR/.../run_kernel_trace.csv reports how much
of the window digests' time overlaps the next windows' scans (the digests run
on their own stream since round 6), and per call when the last
scan ended and when each digest (window digests, the GPU's shares) ran."""
import csv
import glob
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10


def summary(path):
    rows = list(csv.DictReader(open(path)))
    k = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows),
               key=lambda x: x[1])
    # per call (kernels more than 3 ms apart start a new one): when the last
    # scan ended and when each digest ran, in ms from the call's first kernel
    calls, cur = [], [k[0]]
    for x in k[1:]:
        if x[1] - max(e for _, _, e in cur) > 3_000_000:
            calls.append(cur)
            cur = []
        cur.append(x)
    calls.append(cur)
    for i, cl in enumerate(calls):
        c0 = cl[0][1]
        sc = [(s, e) for n, s, e in cl if "scan" in n]
        dg = [(s, e) for n, s, e in cl if "digest" in n and "order" not in n]
        print(f"call {i}: {len(cl)} kernels, {len(sc)} scans, last scan ends "
              f"{((max(e for _, e in sc) - c0) / 1e6) if sc else 0:.2f} ms; digests (start, end) ms: "
              f"{[(round((s - c0) / 1e6, 2), round((e - c0) / 1e6, 2)) for s, e in dg]}")
    scans = [(s, e) for n, s, e in k if "scan" in n]
    digests = [(s, e) for n, s, e in k if "digest" in n and "order" not in n]
    ov = 0
    for ds, de in digests:
        for ss, se in scans:
            ov += max(0, min(de, se) - max(ds, ss))
    dt = sum(e - s for s, e in digests)
    t0 = min(s for _, s, _ in k)
    print(f"scans {len(scans)}, window digests {len(digests)} ({dt / 1e6:.2f} ms), "
          f"scan time inside digest time {ov / 1e6:.3f} ms; digests (start, end) ms from the first "
          f"kernel: {[(round((s - t0) / 1e6, 2), round((e - t0) / 1e6, 2)) for s, e in digests]}; "
          f"last scan ends {(max(e for _, e in scans) - t0) / 1e6:.2f} ms")


def main():
    if sys.argv[1] == "--summary":
        p = sys.argv[2]
        if os.path.isdir(p):
            p = glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)[0]
        summary(p)
        return
    import desync_amd
    gib = float(sys.argv[1])
    n = int(gib * (1 << 30))
    fd, path = tempfile.mkstemp(prefix="dsx_trace_")
    try:
        rng = np.random.default_rng(5)
        with os.fdopen(fd, "wb") as f:
            left = n
            while left:
                k = min(left, 256 << 20)
                f.write(rng.integers(0, 256, k, dtype=np.uint8).tobytes())
                left -= k
            f.flush()
            os.fsync(f.fileno())
        fdr = os.open(path, os.O_RDONLY)
        try:
            desync_amd.index_fd(fdr, MIN, AVG, MAX)  # (warm: context, slots, windows)
            ends, ids = desync_amd.index_fd(fdr, MIN, AVG, MAX)
            print(len(ends), "chunks")
            if "--verify" in sys.argv:  # (then VerifyIndex of the list, twice)
                for _ in range(2):
                    desync_amd.ids_fd(fdr, 0, ends)
        finally:
            os.close(fdr)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
