#!/bin/bash
# A/B of the scan's lane-segment target on the driver's command (config-5
# shard, 8 GiB launches): smaller lane segments = smaller regions = a shorter
# tail after the work queues drain, at the price of more warm-up lines.
# Alternating fresh processes, --no-cpu.  Outputs under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r04d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  for lt in 8448 6336 4224; do
    DSX_LANE_TARGET=$lt timeout -k 10 200 python3 $CMD > $OUT/lane${lt}_$i.json 2> $OUT/lane${lt}_$i.err || { tail $OUT/lane${lt}_$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/lane${lt}_$i.json'));r=d['roofline']
print('lane $lt #$i', d['value'], d['ms_per_step'], r['kernel_ms'], r['clock_mhz'], r.get('wave_busy'), r['scan_share_of_step'])"
  done
done
echo done
