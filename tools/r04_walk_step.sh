#!/bin/bash
# The GPU suite after the walk's chain-step change (next_after32 without the
# per-step range check), then the driver's command under rocprofv3 for the
# stitch kernels' means, and two bench lines.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $CMD > $OUT/trace_bench.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/trace/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('walk', 'fixup', 'gather', 'finish', 'scanl')):
        print(r['Name'][:44], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')"
for i in 1 2; do
  timeout -k 10 200 python3 $CMD > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail $OUT/bench_$i.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/bench_$i.json'));r=d['roofline']
print('bench #$i', d['value'], d['ms_per_step'], r['kernel_ms'], r['clock_mhz'], r.get('wave_busy'), r['scan_share_of_step'])"
done
echo done
