#!/bin/bash
# Shader clock and wave-state counters of the scan per ablation variant
# (0 full, 3 staging only, 4 hashing only), 4 GiB uniform.  The clock is
# GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (kernel trace of the same run).
set -o pipefail
# ablation variants are in the diagnostic build (make -C desync_amd/csrc diag)
export DSX_LIB_PATH=$PWD/desync_amd/libdsx_diag.so
export TMPDIR=/tmp
OUT=gpurun_out/${1:-clk}
mkdir -p $OUT
for v in ${VARS:-0 3 4}; do
  DSX_SCAN_VARIANT=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES -d $OUT/v$v -o run --output-format csv -- python bench.py --gib ${GIB:-4} --steps 5 --warmup 1 --no-cpu > $OUT/v$v.log 2>&1 || exit 1
  echo "== variant $v"
  python tools/pmc_summary.py $OUT/v$v
  python - "$OUT/v$v" <<'EOF'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "scan" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
if d:
    print(f"   scan duration ms: mean {sum(d)/len(d):.4f} (n={len(d)})")
EOF
done
