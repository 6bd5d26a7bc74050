#!/bin/bash
# regions-per-slot sweep for the scan work queue
set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "not config2 and not config4 and not host_and_fd and not exhaustive" > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for r in 1 2 4 8; do
  o=$(DSX_REGIONS_PER_SLOT=$r timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "rps=$r $o"
done
