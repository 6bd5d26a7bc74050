#!/usr/bin/env python3
"""The one A/B tool: bench.py lines under settings, in alternating fresh
processes, optionally with the SMU energy / throttle record of each run.

    python3 tools/ab.py OUTDIR CASE [CASE ...] [--rounds R] [--steps K] [--warmup W]
                        [--smu] [--bench-args "..."] [--timeout S]

A CASE is LABEL:SPEC where SPEC is a comma-separated list of
  VAR=value          an environment setting (DSX_TAIL_SPLIT=3, DSX_SCAN_VARIANT=4, ...)
  diag               run on the diagnostic build (DSX_LIB_PATH=desync_amd/libdsx_diag.so)
  +ARG / +ARG=VAL    an extra bench.py argument (+--inflight=3, +--workload=zeros, +--avg=16)
e.g.   tools/ab.py gpurun_out/x full: v4:diag,DSX_SCAN_VARIANT=4 k3:DSX_TAIL_SPLIT=3 --smu

Round r runs every case once, in order, each in a fresh process (the power
controller's state carries over between cases, so alternation, not blocks, is
what makes two settings comparable).  Every run's bench line is kept under
OUTDIR/LABEL_r.json; with --smu the run goes through tools/smu_sample.py and
OUTDIR/LABEL_r.smu.json holds J/GiB, power, clock and PPT / thermal
residency over the bench's timed window.  The summary (stdout and
OUTDIR/summary.json) gives each case's median, min and max.

Replaces the per-experiment scripts of rounds 2-4 (ab_env.sh, ab_variant.sh,
env_ab.sh, inflight_sweep.sh, smu_bench.sh and the r04_*.sh A/B scripts:
each is one invocation of this tool).
"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DIAG = os.path.join(REPO, "desync_amd", "libdsx_diag.so")
FIELDS = (("value", None), ("ms_per_step", None), ("kernel_ms", "roofline"), ("frac", "roofline"),
          ("clock_mhz", "roofline"), ("wave_busy", "roofline"))
SMU_FIELDS = ("j_per_gib", "j_per_gib_above_idle", "mean_power_w", "gfxclk_mhz_median", "res_ppt",
              "res_socket_thm", "res_vr_thm", "res_hbm_thm", "hotspot_c_max")


def parse_case(text):
    label, _, spec = text.partition(":")
    env, args = {}, []
    for item in filter(None, spec.split(",")):
        if item == "diag":
            env["DSX_LIB_PATH"] = DIAG
        elif item.startswith("+"):
            k, eq, v = item[1:].partition("=")
            args += [k] + ([v] if eq else [])
        else:
            k, _, v = item.partition("=")
            env[k] = v
    return {"label": label, "env": env, "args": args}


def run_case(case, r, a, out):
    tag = f"{case['label']}_{r}"
    bench = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", str(a.steps), "--warmup",
             str(a.warmup), "--no-cpu"] + shlex.split(a.bench_args) + case["args"]
    env = dict(os.environ, **case["env"])
    if a.smu:
        marks = os.path.join(out, tag + ".marks.json")
        cmd = [sys.executable, os.path.join(HERE, "smu_sample.py"), os.path.join(out, tag + ".jsonl"),
               "--"] + bench + ["--marks", marks]
    else:
        cmd = bench
    with open(os.path.join(out, tag + ".json"), "w") as fo, open(os.path.join(out, tag + ".err"), "w") as fe:
        rc = subprocess.call(["timeout", "-k", "10", str(a.timeout)] + cmd, stdout=fo, stderr=fe,
                             env=env, cwd=REPO)
    if rc != 0:
        sys.stdout.write(open(os.path.join(out, tag + ".err")).read()[-3000:])
        raise SystemExit(f"case {tag} failed (exit {rc}): stopping")
    line = json.loads(open(os.path.join(out, tag + ".json")).read().strip().splitlines()[-1])
    row = {k: (line.get(sub) or {}).get(k) if sub else line.get(k) for k, sub in FIELDS}
    if a.smu:
        s = subprocess.run([sys.executable, os.path.join(HERE, "smu_summary.py"),
                            os.path.join(out, tag + ".jsonl"), marks],
                           capture_output=True, text=True, check=True).stdout
        open(os.path.join(out, tag + ".smu.json"), "w").write(s)
        smu = json.loads(s)
        row.update({k: smu.get(k) for k in SMU_FIELDS})
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("cases", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--smu", action="store_true", help="SMU energy / throttle record of each run")
    ap.add_argument("--bench-args", default="", help="bench.py arguments common to every case")
    ap.add_argument("--timeout", type=int, default=240, help="seconds per run")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    cases = [parse_case(c) for c in a.cases]
    rows = {c["label"]: [] for c in cases}
    for r in range(1, a.rounds + 1):
        for c in cases:
            row = run_case(c, r, a, a.out)
            rows[c["label"]].append(row)
            print(f"{c['label']} #{r} " + " ".join(f"{k}={v}" for k, v in row.items() if v is not None),
                  flush=True)
    summary = {}
    for label, rs in rows.items():
        summary[label] = {}
        for k in rs[0]:
            xs = [x[k] for x in rs if isinstance(x.get(k), (int, float))]
            if xs:
                summary[label][k] = {"median": round(statistics.median(xs), 4), "min": min(xs),
                                     "max": max(xs)}
    json.dump({"cases": a.cases, "rounds": a.rounds, "steps": a.steps, "summary": summary},
              open(os.path.join(a.out, "summary.json"), "w"), indent=1)
    for label, s in summary.items():
        print(f"== {label}: " + " ".join(f"{k}={v['median']} [{v['min']}, {v['max']}]"
                                         for k, v in s.items()), flush=True)


if __name__ == "__main__":
    main()
