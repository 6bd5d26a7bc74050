#!/bin/bash
# stitch segment size: walk timeline and repairs per setting
for e in "DSX_SEG_MAX=4" "DSX_SEG_MAX=2 DSX_SEG_FLOOR=0" "DSX_SEG_MAX=1 DSX_SEG_FLOOR=0"; do
  echo "== $e"
  env $e timeout -k 10 60 python tools/scan_trace.py 1 | grep -E "stats|walk|entry|counts|staged" || exit 1
done
