#!/bin/bash
# Scan lane-segment size sweep (DSX_LANE_BYTES) x ablation variants.
set -o pipefail
for lb in ${LBS:-0 528 720 1008 1104 1488 2064 4080}; do
  for v in ${VARS:-0 3}; do
    r=$(DSX_LANE_BYTES=$lb DSX_SCAN_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
    echo "lane_bytes=$lb variant=$v $r"
  done
done
