#!/bin/bash
# A/B of scan settings on the bench line, alternated over rounds:
#   CONFIGS="DSX_SCANM=0 DSX_SCANM=16" ROUNDS=3 bash tools/ab_variant.sh
# (each config is a space-free list of VAR=VALUE pairs joined by ',')
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for cfg in ${CONFIGS:-DSX_SCAN_VARIANT=0 DSX_SCAN_VARIANT=6}; do
    out=$(env ${cfg//,/ } timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} 2>/dev/null) || exit 1
    echo "round=$r $cfg $(echo "$out" | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
