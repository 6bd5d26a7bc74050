#!/bin/bash
# DSX_FUSE (the stitch run as tasks inside the next scans; libdsx_diag.so)
# on the driver's exact command at its default shape (config-5 shard, 8 GiB
# pieces), fresh processes alternating: the diagnostic library with the
# fused stitch off and on (one region size, as the fused path uses), and the
# product library at its defaults.  Outputs under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r04h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
DIAG=$PWD/desync_amd/libdsx_diag.so
for i in 1 2 3; do
  for cfg in "DSX_LIB_PATH=$DIAG,DSX_FUSE=0,DSX_TAIL_SPLIT=0" "DSX_LIB_PATH=$DIAG,DSX_FUSE=1" "DSX_TAIL_SPLIT=3"; do
    tag=$(echo $cfg | sed 's#DSX_LIB_PATH=[^,]*#diag#' | tr '=,' '__')
    env ${cfg//,/ } timeout -k 10 200 python3 $CMD > $OUT/${tag}_$i.json 2> $OUT/${tag}_$i.err || { tail $OUT/${tag}_$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/${tag}_$i.json'));r=d['roofline']
print('$tag #$i', d['value'], d['ms_per_step'], r['kernel_ms'], r['clock_mhz'], r.get('wave_busy'), r['scan_share_of_step'])"
  done
done
echo done
