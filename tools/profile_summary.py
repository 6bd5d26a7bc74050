#!/usr/bin/env python3
"""One-page summary of a closing profile directory written by
tools/r04_final.sh (gpurun_out/<tag>/ or profiles/<tag>/): the bench lines,
the stamped scan against rocprofv3's timed dispatches, traffic, configs 3/4,
chunk-ID and file rates, the CPU baseline.

usage: profile_summary.py DIR [--write]   (--write: DIR/SUMMARY.txt as well)
"""
import csv
import json
import os
import sys


def load(d, name):
    p = os.path.join(d, name)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def bench_line(name, b):
    r = b.get("roofline") or {}
    keys = ("kernel_ms", "kernel_ms_min_max", "frac", "clock_mhz", "wave_busy", "scan_share_of_step")
    return f"{name:22s} {b['value']:9.2f} GiB/s  {b['ms_per_step']:.4f} ms/step  " + \
        " ".join(f"{k}={r.get(k)}" for k in keys if k in r)


def main():
    d = sys.argv[1]
    out = []
    for name in ("bench.json", "bench_2.json", "bench_nostamps.json", "trace_bench.json",
                 "bench_dedup.json", "bench_zeros.json"):
        b = load(d, name)
        if b:
            out.append(bench_line(name, b))
    b = load(d, "bench.json")
    if b and "cpu_baseline" in b:
        c = b["cpu_baseline"]
        out.append(f"cpu_baseline {c['value']} GiB/s on {c['cores']} threads; n=10 {c.get('n10_gibs')}; "
                   f"1 thread {c.get('single_thread_gibs')}; IDs {c.get('ids_sha512_256_gibs')}")
    trace = None
    for sub in ("trace/run_kernel_trace.csv", "trace_kernel_trace.csv"):
        if os.path.exists(os.path.join(d, sub)):
            trace = os.path.join(d, sub)
            break
    if trace:
        rows = [r for r in csv.DictReader(open(trace)) if "scanl_kernel" in r["Kernel_Name"]]
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
        if ms:
            out.append(f"rocprofv3 scanl_kernel: {len(ms)} dispatches, mean {sum(ms) / len(ms):.4f} ms, "
                       f"timed last 80 {sum(ms[-80:]) / min(80, len(ms)):.4f} ms")
    for sub in ("trace/run_kernel_stats.csv", "kernel_stats_bench.csv"):
        p = os.path.join(d, sub)
        if os.path.exists(p):
            for r in csv.DictReader(open(p)):
                if any(k in r["Name"] for k in ("scanl", "walk", "fixup", "gather", "finish", "publish")):
                    out.append(f"  {r['Name'][:50]:50s} calls {r['Calls']:>4s} mean {float(r['AverageNs']) / 1e3:8.1f} us")
            break
    t = load(d, "traffic_uniform_8589934592.json")
    if t:
        out.append(f"HBM reads per 8 GiB scan: {t['hbm_bytes_per_launch']:.0f} B = {t['ratio_to_input']:.4f} x input")
    g = load(d, "digest_rate.json")
    if g:
        for r in g["rows"]:
            out.append("ids " + str(r["gib"]) + " GiB: " +
                       ", ".join(f"{k} {v}" for k, v in r.items() if k.endswith("_gibs")))
    m = load(d, "make_rate.json")
    if m:
        for r in m["rows"]:
            out.append(f"file {r['gib']} GiB: " + ", ".join(
                f"{k} {r[k]['gibs_median']} ({r[k]['gibs_min']}-{r[k]['gibs_max']})"
                for k in ("make", "index_fd", "cut_fd", "verify") if k in r))
    text = "\n".join(out)
    print(text)
    if "--write" in sys.argv:
        with open(os.path.join(d, "SUMMARY.txt"), "w") as f:
            f.write(f"# tools/profile_summary.py {os.path.basename(os.path.normpath(d))}\n" + text + "\n")


if __name__ == "__main__":
    main()
