#!/bin/bash
# Chunk-ID rates with the block prefetch on (2 waves per SIMD for SHA-512)
# and off (3 waves per SIMD), longest-first order at every size.
# Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for pf in 1 0; do
  DSX_DIGEST_PF=$pf timeout -k 10 400 python3 tools/digest_rate.py 1 4 16 > $OUT/digest_rate_pf$pf.json 2> $OUT/digest_rate_pf$pf.err || { tail $OUT/digest_rate_pf$pf.err; exit 1; }
  python3 -c "
import json
for r in json.load(open('$OUT/digest_rate_pf$pf.json'))['rows']:
    print('pf=$pf', r['gib'], {k: v for k, v in r.items() if k.endswith('_gibs')})"
done

for pf in 1 0; do
  DSX_DIGEST_PF=$pf DSX_RATE_REPS=3 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_digest_pf$pf -o run --output-format csv -- python3 tools/digest_rate.py 16 > $OUT/trace_digest_pf$pf.log 2>&1 || { tail $OUT/trace_digest_pf$pf.log; exit 1; }
done
echo traced
