#!/bin/bash
# quick scan-geometry sweep: prints variant, lane bytes, scan kernel ms
for v in ${VARIANTS:-3 0}; do
  for s in ${LANES:-768 1536 3072 8208}; do
    r=$(DSX_SCAN_VARIANT=$v DSX_LANE_BYTES=$s timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*' | tr '\n' ' ')
    echo "variant=$v S=$s $r"
  done
done
