#!/bin/bash
# Runs bench.py once per environment setting given as arguments
# (e.g. "DSX_PREFETCH=2 DSX_SCAN_CFG=0"); prints value / kernel_ms per line.
set -o pipefail
for e in "$@"; do
  r=$(env $e timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "$e :: $r"
done
