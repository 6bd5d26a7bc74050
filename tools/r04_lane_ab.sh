#!/bin/bash
# A/B of the scan's region granularity on the driver's command (config-5
# shard, 8 GiB launches): the default lane segments (8448 B), shorter lane
# segments everywhere (DSX_LANE_TARGET), or short ones only for the tail
# regions (DSX_TAIL_SPLIT=k: two region sizes; DSX_TAIL_MULT=j: how much of
# the piece is tail).  Alternating fresh processes, --no-cpu.
#   tools/r04_lane_ab.sh TAG [CONFIG ...]   (a CONFIG is "VAR=v[,VAR=v]")
# Outputs under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r04d}; shift
CFGS=("$@")
[ ${#CFGS[@]} -gt 0 ] || CFGS=("DSX_TAIL_SPLIT=0" "DSX_TAIL_SPLIT=4" "DSX_TAIL_SPLIT=2" "DSX_LANE_TARGET=6336")
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  for cfg in "${CFGS[@]}"; do
    tag=$(echo $cfg | tr '=,' '__')
    env ${cfg//,/ } timeout -k 10 200 python3 $CMD > $OUT/${tag}_$i.json 2> $OUT/${tag}_$i.err || { tail $OUT/${tag}_$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/${tag}_$i.json'));r=d['roofline']
print('$cfg #$i', d['value'], d['ms_per_step'], r['kernel_ms'], r['clock_mhz'], r.get('wave_busy'), r['scan_share_of_step'])"
  done
done
echo done
