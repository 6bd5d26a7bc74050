#!/bin/bash
# L2 prefetch distance sweep (DSX_PREFETCH batches), scan config 0
set -o pipefail
for pf in ${PFS:-0 2 4 8}; do
for v in ${VARS:-0 3}; do
  o=$(DSX_PREFETCH=$pf DSX_SCAN_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "pf=$pf variant=$v $o"
done
done
