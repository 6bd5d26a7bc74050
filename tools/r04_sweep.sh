#!/bin/bash
# SURVEY.md 8(d)'s average-size sweep (min = avg/4, max = 4 avg; 16/64/256 KiB)
# on the driver's command shape, plus the two-region-size edge tests.
# Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "two_region" -x -v --timeout 240 --timeout-method thread > $OUT/pytest_edges.log 2>&1 || { tail -30 $OUT/pytest_edges.log; exit 1; }
tail -4 $OUT/pytest_edges.log
for i in 1 2; do
  for avg in 16 64 256; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --avg $avg > $OUT/avg${avg}_$i.json 2> $OUT/avg${avg}_$i.err || { tail $OUT/avg${avg}_$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/avg${avg}_$i.json'));r=d['roofline']
print('avg $avg #$i', d['value'], d['ms_per_step'], d['config']['chunks'], r['kernel_ms'], r['clock_mhz'], r.get('wave_busy'), r['scan_share_of_step'])"
  done
done
echo done
