#!/usr/bin/env python3
"""Summarise tools/smu_sample.py output over a bench's timed window.

    python3 tools/smu_summary.py SAMPLES.jsonl [MARKS.json]

MARKS.json is what `bench.py --marks` writes: {"t0", "t1", "bytes"} (unix
time around the timed steps, bytes chunked in them).  Without it the window
is every sample whose socket power exceeds 2x the idle median.

Reports, over the window: energy from the SMU's energy accumulator (and the
integral of current_socket_power as a cross-check), mean power, J/GiB total
and above idle, the median gfx clock, and the residency of each throttle /
violation reason (PPT = package power limit, socket / VR / HBM thermal,
PROCHOT) as a fraction of the window, from the SMU's own accumulators.
"""
import json
import statistics
import sys

GiB = float(1 << 30)


def load(path):
    static, rows = {}, []
    for line in open(path):
        d = json.loads(line)
        if "static" in d:
            static = d["static"]
        elif "t" in d:
            rows.append(d)
    return static, rows


def interp(rows, key, t):
    """Value of a monotone accumulator at time t (linear between samples)."""
    pts = [(r["t"], r[key]) for r in rows if isinstance(r.get(key), (int, float))]
    if not pts:
        return None
    if t <= pts[0][0]:
        return pts[0][1]
    for (ta, va), (tb, vb) in zip(pts, pts[1:]):
        if ta <= t <= tb:
            return va if tb == ta else va + (vb - va) * (t - ta) / (tb - ta)
    return pts[-1][1]


def viol_at(rows, key, t):
    pts = [(r["t"], r["viol"].get(key)) for r in rows if "viol" in r]
    pts = [(a, b) for a, b in pts if isinstance(b, (int, float))]
    best = None
    for a, b in pts:
        if best is None or abs(a - t) < abs(best[0] - t):
            best = (a, b)
    return best


def med(xs):
    xs = [x for x in xs if isinstance(x, (int, float))]
    return round(statistics.median(xs), 1) if xs else None


def summarise(static, rows, marks=None):
    res = static.get("energy", {})
    unit = res.get("counter_resolution") if isinstance(res, dict) else None
    unit_j = (unit or 15.259) * 1e-6  # uJ per count
    t_start = rows[0]["t"]
    idle_rows = [r for r in rows if r["t"] < t_start + 0.25]
    p_idle = med(r.get("current_socket_power") for r in idle_rows)
    if marks:
        t0, t1, nbytes = marks["t0"], marks["t1"], marks.get("bytes")
    else:
        busy = [r for r in rows if (r.get("current_socket_power") or 0) > 2 * (p_idle or 1e9)]
        t0, t1, nbytes = busy[0]["t"], busy[-1]["t"], None
    win = [r for r in rows if t0 <= r["t"] <= t1]
    dt = t1 - t0
    e0, e1 = interp(rows, "energy_accumulator", t0), interp(rows, "energy_accumulator", t1)
    energy = (e1 - e0) * unit_j if e0 is not None and e1 is not None else None
    # integral of current_socket_power (W) over the window, as a cross-check
    pw = [(r["t"], r["current_socket_power"]) for r in win
          if isinstance(r.get("current_socket_power"), (int, float))]
    e_int = sum((b[0] - a[0]) * a[1] for a, b in zip(pw, pw[1:])) if len(pw) > 1 else None
    distinct_e = len({r.get("energy_accumulator") for r in win})
    out = {
        "bdf": static.get("bdf"), "power_cap": static.get("power_cap"),
        "window_s": round(dt, 4), "samples": len(win), "distinct_energy_values": distinct_e,
        "idle_w": p_idle,
        "energy_j": round(energy, 3) if energy is not None else None,
        "mean_power_w": round(energy / dt, 1) if energy and dt > 0 else None,
        "power_integral_j": round(e_int, 3) if e_int else None,
        "current_socket_power_w_median": med(r.get("current_socket_power") for r in win),
        "current_socket_power_w_max": max((r.get("current_socket_power") or 0 for r in win), default=None),
        "average_socket_power_w_median": med(r.get("average_socket_power") for r in win),
        "gfxclk_mhz_median": med(r.get("current_gfxclk") for r in win),
        "avg_gfxclk_mhz_median": med(r.get("average_gfxclk_frequency") for r in win),
        "uclk_mhz_median": med(r.get("current_uclk") for r in win),
        "hotspot_c_max": max((r.get("temperature_hotspot") or 0 for r in win), default=None),
        "hbm_c_max": max((r.get("temperature_mem") or 0 for r in win), default=None),
        "vrgfx_c_max": max((r.get("temperature_vrgfx") or 0 for r in win), default=None),
        "voltage_gfx_mv_median": med(r.get("voltage_gfx") for r in win),
        "throttle_status_seen": sorted({r.get("throttle_status") for r in win} - {None}, key=str),
        "indep_throttle_status_seen": sorted({r.get("indep_throttle_status") for r in win} - {None}, key=str),
    }
    clks = [r.get("current_gfxclks") for r in win if isinstance(r.get("current_gfxclks"), list)]
    if clks:
        n = max(len(c) for c in clks)
        out["gfxclk_per_xcc_median"] = [med(c[i] for c in clks if i < len(c)
                                             and isinstance(c[i], (int, float))) for i in range(n)]
    if nbytes:
        out["gib"] = round(nbytes / GiB, 3)
        if energy:
            out["j_per_gib"] = round(energy / (nbytes / GiB), 4)
            if p_idle:
                out["j_per_gib_above_idle"] = round((energy - p_idle * dt) / (nbytes / GiB), 4)
    # residency accumulators in gpu_metrics: each counts the SMU's sampling
    # ticks (accumulation_counter) spent with that limit active
    ac0, ac1 = interp(rows, "accumulation_counter", t0), interp(rows, "accumulation_counter", t1)
    if ac0 is not None and ac1 is not None and ac1 > ac0:
        for k in ("ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc",
                  "hbm_thm_residency_acc", "prochot_residency_acc"):
            a, b = interp(rows, k, t0), interp(rows, k, t1)
            if a is not None and b is not None:
                out["res_" + k.replace("_residency_acc", "")] = round((b - a) / (ac1 - ac0), 4)
        out["accumulation_ticks"] = ac1 - ac0
    # violation status accumulators (amdsmi_get_violation_status)
    c0, c1 = viol_at(rows, "acc_counter", t0), viol_at(rows, "acc_counter", t1)
    if c0 and c1 and c1[1] > c0[1]:
        for k in ("acc_ppt_pwr", "acc_socket_thrm", "acc_vr_thrm", "acc_hbm_thrm",
                  "acc_prochot_thrm", "acc_gfx_clk_below_host_limit"):
            a, b = viol_at(rows, k, t0), viol_at(rows, k, t1)
            if a and b:
                out["viol_" + k[4:]] = round((b[1] - a[1]) / (c1[1] - c0[1]), 4)
        out["viol_ticks"] = c1[1] - c0[1]
    return out


def main():
    static, rows = load(sys.argv[1])
    marks = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else None
    print(json.dumps(summarise(static, rows, marks)))


if __name__ == "__main__":
    main()
