#!/bin/bash
# rocprofv3 kernel trace of serial bench jobs; prints the last jobs' kernel
# durations and the gaps between them
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tl}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python bench.py --no-cpu --inflight 1 --steps ${STEPS:-8} --warmup 2 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/err || { tail $OUT/err; exit 1; }
python - $OUT <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-14:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0
    print(f"{r['Kernel_Name'][:34]:34s} dur {(e - s) / 1000:8.1f} us  gap {gap:7.1f}")
    prev = e
PY
