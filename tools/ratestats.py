"""Repeat-and-summarise helper of the rate tools (measurement hygiene: every
point is timed REPS times and reported as median with min / max, not best)."""
import os
import statistics
import time

REPS = int(os.environ.get("DSX_RATE_REPS", "10"))


def repeat(fn, nbytes, reps=None, warmup=1):
    """Times fn() `reps` times after `warmup` untimed calls; returns (summary
    dict in GiB/s and s, the last result)."""
    reps = reps or REPS
    r = None
    for _ in range(warmup):
        r = fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    g = nbytes / (1 << 30)
    return {"gibs_median": round(g / med, 2), "gibs_min": round(g / max(ts), 2),
            "gibs_max": round(g / min(ts), 2), "s_median": round(med, 5), "reps": reps}, r
