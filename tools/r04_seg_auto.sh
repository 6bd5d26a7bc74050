#!/bin/bash
# The GPU suite with the segment-size rule (DSX_SEG_TARGET=4096: 2 MiB stitch
# segments on 8 GiB pieces), then the rule against 1 MiB segments
# (DSX_SEG_TARGET=0) on the driver's command, fresh processes alternating.
# Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash tools/r04_lane_ab.sh $TAG DSX_SEG_TARGET=4096 DSX_SEG_TARGET=0 || exit 1
