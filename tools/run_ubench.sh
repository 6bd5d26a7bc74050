#!/bin/bash
# Runs the staging / VALU microbenchmarks (built in-tree beforehand) on the
# GPU box; output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
if [ -x tools/ubench_staging ]; then
  timeout -k 10 300 ./tools/ubench_staging ${GIB:-4} > gpurun_out/ubench_staging.txt 2>&1 || exit 1
  cat gpurun_out/ubench_staging.txt
fi
if [ -x tools/ubench_valu ] && [ -n "$VALU" ]; then
  timeout -k 10 300 ./tools/ubench_valu > gpurun_out/ubench_valu.txt 2>&1 || exit 1
  cat gpurun_out/ubench_valu.txt
fi
