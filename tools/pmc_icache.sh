#!/bin/bash
# instruction-cache and instruction-mix counters of the scan (1 GiB)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ic}
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INSTS_VALU -d $OUT/p -o run --output-format csv -- python bench.py --gib ${GIB:-1} --steps 5 --warmup 1 --no-cpu --inflight 1 > $OUT/p.log 2>&1 || exit 1
python tools/pmc_summary.py $OUT/p
