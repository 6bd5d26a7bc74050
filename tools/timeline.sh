#!/bin/bash
# rocprofv3 kernel trace of serial bench jobs; prints the last jobs' kernel
# durations and the gaps between them
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tl}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python bench.py --no-cpu --inflight ${INFLIGHT:-1} --steps ${STEPS:-8} --warmup 2 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/err || { tail $OUT/err; exit 1; }
python - $OUT <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
import os
n = int(os.environ.get("ROWS", "14"))
skip = int(os.environ.get("SKIP", "0"))  # rows to leave out at the end (the serial pass)
sel = rows[-n - skip:len(rows) - skip]
t0 = int(sel[0]["Start_Timestamp"])
prev = None
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0
    print(f"{r['Kernel_Name'][:34]:34s} q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3} "
          f"start {(s - t0) / 1000:8.1f} dur {(e - s) / 1000:8.1f} us  gap {gap:7.1f}")
    prev = max(prev or 0, e)
PY
