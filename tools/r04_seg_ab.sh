#!/bin/bash
# Stitch segment size on the driver's command (DSX_SEG_FLOOR: 1 MiB default,
# 2, 4, 8 MiB): bench lines in alternating fresh processes, then one
# rocprofv3 --kernel-trace --stats pass per size for the stitch kernels.
# Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  for f in 1048576 2097152 4194304 8388608; do
    DSX_SEG_FLOOR=$f timeout -k 10 200 python3 $CMD > $OUT/seg${f}_$i.json 2> $OUT/seg${f}_$i.err || { tail $OUT/seg${f}_$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/seg${f}_$i.json'));r=d['roofline']
print('seg $f #$i', d['value'], d['ms_per_step'], d['config']['chunks'], r['kernel_ms'], r['clock_mhz'], r.get('wave_busy'), r['scan_share_of_step'])"
  done
done
for f in 1048576 2097152 4194304 8388608; do
  DSX_SEG_FLOOR=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_seg$f -o run --output-format csv -- python3 $CMD > $OUT/trace_seg$f.json 2> $OUT/trace_seg$f.err || { tail $OUT/trace_seg$f.err; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/trace_seg$f/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('walk', 'fixup', 'gather', 'finish', 'publish', 'scanl')):
        print('seg $f', r['Name'][:44], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')"
done
echo done
