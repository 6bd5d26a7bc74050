#!/bin/bash
# Power / clock / throttle evidence for the bench's own job:
#   tools/smu_bench.sh OUTDIR STEPS [LABEL:ENV:ARGS ...]
# Each case runs `bench.py --steps STEPS --warmup 5 --no-cpu` under
# tools/smu_sample.py (SMU energy accumulator, power, clocks, throttle and
# violation residency at ~2 ms), with the bench's timed window written by
# --marks, and is summarised by tools/smu_summary.py into OUTDIR/LABEL.smu.json.
# ENV is a space-separated list of VAR=VALUE (may be empty); ARGS extra bench
# arguments.  Example:
#   tools/smu_bench.sh gpurun_out/r05a 300 full:: v3:"DSX_LIB_PATH=$PWD/desync_amd/libdsx_diag.so DSX_SCAN_VARIANT=3":
set -o pipefail
OUT=$1; STEPS=$2; shift 2
mkdir -p "$OUT"
for case in "$@"; do
  label=${case%%:*}; rest=${case#*:}; envs=${rest%%:*}; args=${rest#*:}
  echo "== $label env=[$envs] args=[$args]"
  env $envs timeout -k 10 240 python3 tools/smu_sample.py "$OUT/$label.jsonl" -- \
      python3 bench.py --steps "$STEPS" --warmup 5 --no-cpu --marks "$OUT/$label.marks.json" $args \
      > "$OUT/$label.bench.json" 2> "$OUT/$label.err" || { echo "case $label failed"; tail -5 "$OUT/$label.err"; exit 1; }
  python3 tools/smu_summary.py "$OUT/$label.jsonl" "$OUT/$label.marks.json" > "$OUT/$label.smu.json" || exit 1
  python3 - "$OUT/$label.bench.json" "$OUT/$label.smu.json" <<'EOF'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = json.load(open(sys.argv[2]))
r = b.get("roofline", {})
keys = ("window_s", "idle_w", "mean_power_w", "current_socket_power_w_median", "current_socket_power_w_max",
        "gfxclk_mhz_median", "j_per_gib", "j_per_gib_above_idle", "hotspot_c_max", "throttle_status_seen",
        "res_ppt", "res_socket_thm", "res_vr_thm", "res_hbm_thm", "viol_ppt_pwr", "viol_socket_thrm",
        "viol_vr_thrm", "viol_gfx_clk_below_host_limit", "power_cap")
print(f"  value {b['value']} GiB/s  scan {r.get('kernel_ms')} ms  frac {r.get('frac')}  clock {r.get('clock_mhz')}  "
      + " ".join(f"{k}={s.get(k)}" for k in keys))
EOF
done
