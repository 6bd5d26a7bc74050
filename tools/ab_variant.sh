#!/bin/bash
# A/B of scan settings on the bench line, alternated over rounds:
#   CONFIGS="DSX_LANE_TARGET=8448 DSX_LANE_TARGET=2304" ROUNDS=3 bash tools/ab_variant.sh
# (each config is a space-free list of VAR=VALUE pairs joined by ',')
# (ablation / trace variants live in the diagnostic build: DIAG=1 loads
# desync_amd/libdsx_diag.so, built beforehand with make -C desync_amd/csrc diag)
set -o pipefail
mkdir -p gpurun_out
[ "${DIAG:-0}" = 1 ] && export DSX_LIB_PATH=$PWD/desync_amd/libdsx_diag.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for cfg in ${CONFIGS:-DSX_SCAN_VARIANT=0 DSX_SCAN_VARIANT=6}; do
    out=$(env ${cfg//,/ } timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} 2>/dev/null) || exit 1
    echo "round=$r $cfg $(echo "$out" | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
