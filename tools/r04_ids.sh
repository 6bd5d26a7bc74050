#!/bin/bash
# Round-4 chunk-ID and host-pipeline measurements: digest rates with the
# longest-first queue on and off, the digest kernel's SQ counters at 16 GiB,
# and the IndexFromFile / VerifyIndex rates.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 tools/digest_rate.py 1 4 16 > $OUT/digest_rate.json 2> $OUT/digest_rate.err || { tail $OUT/digest_rate.err; exit 1; }
cat $OUT/digest_rate.json
DSX_DIGEST_LPT=0 timeout -k 10 400 python3 tools/digest_rate.py 4 16 > $OUT/digest_rate_nolpt.json 2> $OUT/digest_rate_nolpt.err || { tail $OUT/digest_rate_nolpt.err; exit 1; }
cat $OUT/digest_rate_nolpt.json
for lpt in 1 0; do
  DSX_DIGEST_LPT=$lpt DSX_RATE_REPS=2 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/pmc_digest_lpt$lpt -o run --output-format csv -- python3 tools/digest_rate.py 16 > $OUT/pmc_digest_lpt$lpt.log 2>&1 || { tail $OUT/pmc_digest_lpt$lpt.log; exit 1; }
done
timeout -k 10 600 python3 tools/make_rate.py 1 4 > $OUT/make_rate.json 2> $OUT/make_rate.err || { tail $OUT/make_rate.err; exit 1; }
cat $OUT/make_rate.json
echo done
