#!/bin/bash
# Instruction-cache and instruction-mix counters of the scan, one counter
# group per rocprofv3 pass:  tools/pmc_icache.sh OUTDIR [bench args...]
# (e.g. --avg 16 --gib 8).  Summaries via tools/pmc_summary.py.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ic}; shift
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d $OUT/ic -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu "$@" > $OUT/ic.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/mix -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu "$@" > $OUT/mix.log 2>&1 || exit 1
python3 tools/pmc_summary.py $OUT/ic
python3 tools/pmc_summary.py $OUT/mix
