#!/bin/bash
# (fuse_power.sh: DSX_FUSE=1/0 bench lines under board-power sampling)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fpow}
mkdir -p $OUT
for f in 1 0 1 0; do
  DSX_FUSE=$f timeout -k 10 200 tools/power_sample.sh $OUT/pw$f.txt -- python bench.py --no-cpu --warmup 300 --steps 2000 > $OUT/b$f.json 2> $OUT/b$f.err || { tail $OUT/b$f.err; exit 1; }
  echo "fuse=$f $(python -c "import json;d=json.load(open('$OUT/b$f.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])") $(python tools/power_summary.py $OUT/pw$f.txt)"
done
