#!/usr/bin/env python3
"""Summarise tools/power_sample.sh output: the busiest GPU's power, shader
clock and temperature while it draws more than 2x its idle power."""
import json
import statistics
import sys

rows = [l.split() for l in open(sys.argv[1]) if l.strip()]
ng = (len(rows[0]) - 1) // 3


def col(g, k):
    return [float(r[1 + 3 * g + k]) if r[1 + 3 * g + k] != "-" else float("nan") for r in rows]


g = max(range(ng), key=lambda i: max(col(i, 0)))
p, f, t = col(g, 0), col(g, 1), col(g, 2)
idle = min(p)
busy = [i for i in range(len(rows)) if p[i] > 2 * idle]
out = {"samples": len(rows), "busy_samples": len(busy), "idle_w": round(idle / 1e6, 1)}
if busy:
    out.update({
        "busy_power_w_median": round(statistics.median(p[i] for i in busy) / 1e6, 1),
        "busy_power_w_max": round(max(p[i] for i in busy) / 1e6, 1),
        "busy_sclk_mhz_median": round(statistics.median(f[i] for i in busy) / 1e6),
        "busy_temp_c_max": round(max(t[i] for i in busy) / 1e3, 1),
        "busy_s": round(float(rows[busy[-1]][0]) - float(rows[busy[0]][0]), 3),
    })
print(json.dumps(out))
