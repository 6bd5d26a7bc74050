#!/bin/bash
# bench.py per (env setting, GiB) pair; prints value / kernel_ms / stitch_ms
set -o pipefail
for g in ${GIBS:-1 4}; do
for e in "$@"; do
  r=$(env $e timeout -k 10 120 python bench.py --gib $g --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "gib=$g $e :: $r"
done
done
