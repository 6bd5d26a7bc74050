#!/bin/bash
# bench value per jobs-in-flight setting, interleaved twice
set -o pipefail
for rep in 1 2; do
for k in ${KS:-2 3 4 6}; do
  r=$(timeout -k 10 120 python bench.py --no-cpu --inflight $k 2>/dev/null | grep -o '"value": [0-9.]*') || exit 1
  echo "inflight=$k $r"
done
done
