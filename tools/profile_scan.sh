#!/bin/bash
# Profiling recipe for the scan kernel (run on the GPU box from the repo root):
#   kernel-trace stats + PMC passes (one counter group per pass; never with
#   --sys-trace/--runtime-trace).  Outputs under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-prof}
STEPS=${STEPS:-8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="python bench.py --steps $STEPS --warmup 2 --no-cpu ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || exit 1
i=0
for grp in "${@:2}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- $B > $OUT/pmc$i.log 2>&1 || exit 1
done
