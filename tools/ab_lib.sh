#!/bin/bash
# A/B: base vs new library, alternating
set -o pipefail
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-4}); do
  for lib in libdsx_base.so libdsx.so; do
    out=$(DSX_LIB_PATH=$PWD/desync_amd/$lib timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu 2>/dev/null) || exit 1
    echo "round=$r $lib $(echo "$out" | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
