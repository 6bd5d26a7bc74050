#!/bin/bash
# kernel timeline of queued bench jobs with an empty kernel before each scan
# (diagnostic build): where the idle gap between jobs sits
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-gap}
mkdir -p $OUT
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_NOOP_BEFORE_SCAN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python bench.py --no-cpu --steps 60 --warmup 20 > $OUT/b.json 2> $OUT/err.txt || { tail $OUT/err.txt; exit 1; }
python - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/t/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
out = [(r["Kernel_Name"][:26], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
prev = None
base = out[200][1]
for n, s, e in out[200:216]:
    print(f"{n:28s} start {(s-base)/1000:8.1f} dur {(e-s)/1000:6.1f} gap {(s-prev)/1000 if prev else 0:5.1f}")
    prev = e
PY
