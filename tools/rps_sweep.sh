#!/bin/bash
# regions-per-slot x variant sweep for one scan config (CFG, default 0)
set -o pipefail
for r in ${RPS:-1 4}; do
for v in ${VARS:-0 3 4}; do
  o=$(DSX_SCAN_CFG=${CFG:-0} DSX_SCAN_VARIANT=$v DSX_REGIONS_PER_SLOT=$r timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "cfg=${CFG:-0} rps=$r variant=$v $o"
done
done
