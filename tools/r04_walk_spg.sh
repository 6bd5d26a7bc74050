#!/bin/bash
# Segments per walk workgroup (DSX_WALK_SPG caps the automatic 8 for an
# 8 GiB piece in 2 MiB segments): phase 1 walks spg + 1 chains over 4 waves,
# so spg = 7 takes two rounds instead of three and spg = 3 one.  Bench lines
# alternating, then rocprofv3 kernel means.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
bash tools/r04_lane_ab.sh $TAG DSX_WALK_SPG=0 DSX_WALK_SPG=7 DSX_WALK_SPG=3 || exit 1
for f in 0 7 3; do
  DSX_WALK_SPG=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_spg$f -o run --output-format csv -- python3 $CMD > $OUT/trace_spg$f.json 2> $OUT/trace_spg$f.err || { tail $OUT/trace_spg$f.err; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/trace_spg$f/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('walk', 'fixup', 'gather', 'finish')):
        print('spg $f', r['Name'][:44], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')"
done
echo done
