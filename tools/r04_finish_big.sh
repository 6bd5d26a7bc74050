#!/bin/bash
# finish_kernel over up to 4352 segments (an 8 GiB piece in 2 MiB segments:
# K3 + K4 in one multi-workgroup launch) against fixup_fast_kernel +
# gather_kernel (DSX_FINISH_BIG=0) on the driver's command, after the GPU
# suite; then rocprofv3 kernel means of both.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash tools/r04_lane_ab.sh $TAG DSX_FINISH_BIG=1 DSX_FINISH_BIG=0 || exit 1
for f in 1 0; do
  DSX_FINISH_BIG=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_fb$f -o run --output-format csv -- python3 $CMD > $OUT/trace_fb$f.json 2> $OUT/trace_fb$f.err || { tail $OUT/trace_fb$f.err; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/trace_fb$f/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('walk', 'fixup', 'gather', 'finish', 'publish', 'scanl')):
        print('finish_big $f', r['Name'][:44], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')"
done
echo done
