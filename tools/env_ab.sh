#!/bin/bash
# bench kernel_ms / ms_per_step under env settings: each arg is "NAME=VAL,NAME=VAL"
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fenv}
mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $(echo $cfg | tr ',' ' ') timeout -k 10 200 python bench.py --no-cpu > $OUT/b$i.json 2> $OUT/b$i.err || { tail $OUT/b$i.err; exit 1; }
  echo "$cfg $(python -c "import json;d=json.load(open('$OUT/b$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['stitch_ms'])")"
done
