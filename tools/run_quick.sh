#!/bin/bash
# quick GPU check: parity subset + bench for the scan configs / ablations
#   CFGS="cfg:variant ..." (DSX_SCAN_CFG, DSX_SCAN_VARIANT)
set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "not config2 and not config4 and not host_and_fd and not exhaustive" > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -2 gpurun_out/q_tests.log
for cv in ${CFGS:-0:0 1:0 2:0 1:1 1:3}; do
  c=${cv%:*}; v=${cv#*:}
  r=$(DSX_SCAN_CFG=$c DSX_SCAN_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "cfg=$c variant=$v $r"
done
