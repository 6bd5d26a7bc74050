#!/bin/bash
# A round's closing profile on the GPU box, outputs under gpurun_out/$TAG/:
#   the GPU suite; the driver's command under the SMU sampler (energy, clock,
#   PPT / thermal residency: tools/smu_sample.py); again without the stamps;
#   under rocprofv3 --kernel-trace --stats; an L2 read-request --pmc pass (HBM
#   bytes per launch) and a GRBM_GUI_ACTIVE / SQ_BUSY_CYCLES pass; the dedup
#   and zeros workloads; chunk-ID, IndexFromFile / VerifyIndex and streaming
#   rates; the --avg 16 / 64 / 256 sweep (tools/ab.py, alternating processes).
#   tools/profile_summary.py condenses it into SUMMARY.txt.
#   tools/round_profile.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python3 tools/smu_sample.py $OUT/smu_bench.jsonl -- python3 $CMD --marks $OUT/bench.marks.json > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 tools/smu_summary.py $OUT/smu_bench.jsonl $OUT/bench.marks.json > $OUT/smu_bench.json && cat $OUT/smu_bench.json
timeout -k 10 200 python3 $CMD --no-cpu > $OUT/bench_2.json 2> $OUT/bench_2.err || { tail $OUT/bench_2.err; exit 1; }
DSX_BENCH_STAMPS=0 timeout -k 10 200 python3 $CMD --no-cpu > $OUT/bench_nostamps.json 2> $OUT/bench_nostamps.err || { tail $OUT/bench_nostamps.err; exit 1; }
echo "again: $(cat $OUT/bench_2.json)"; echo "no stamps: $(cat $OUT/bench_nostamps.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $CMD > $OUT/trace_bench.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
cat $OUT/trace_bench.json
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/pmc_rdreq -o run --output-format csv -- python3 $CMD --no-cpu > $OUT/pmc_rdreq.json 2> $OUT/pmc_rdreq.err || { tail $OUT/pmc_rdreq.err; exit 1; }
python3 tools/traffic_json.py $OUT/pmc_rdreq 8589934592 uniform > $OUT/traffic_uniform_8589934592.json && cat $OUT/traffic_uniform_8589934592.json
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $OUT/pmc_clk -o run --output-format csv -- python3 $CMD --no-cpu > $OUT/pmc_clk.json 2> $OUT/pmc_clk.err || { tail $OUT/pmc_clk.err; exit 1; }
for w in dedup zeros; do
  timeout -k 10 300 python3 $CMD --workload $w --no-cpu > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail $OUT/bench_$w.err; exit 1; }
  echo "$w: $(cat $OUT/bench_$w.json)"
done
timeout -k 10 400 python3 tools/digest_rate.py 1 4 16 > $OUT/digest_rate.json 2> $OUT/digest_rate.err || { tail $OUT/digest_rate.err; exit 1; }
timeout -k 10 600 python3 tools/make_rate.py 1 2 4 > $OUT/make_rate.json 2> $OUT/make_rate.err || { tail $OUT/make_rate.err; exit 1; }
timeout -k 10 300 python3 tools/stream_rate.py > $OUT/stream_rate.json 2> $OUT/stream_rate.err || { tail $OUT/stream_rate.err; exit 1; }
timeout -k 10 600 python3 tools/ab.py --rounds 3 $OUT/avg 'a16:+--avg=16' 'a64:+--avg=64' 'a256:+--avg=256' > $OUT/avg_sweep.txt 2>&1 || { tail $OUT/avg_sweep.txt; exit 1; }
grep "^==" $OUT/avg_sweep.txt
python3 -c "
import json
for r in json.load(open('$OUT/digest_rate.json'))['rows']: print('ids', r['gib'], {k: v for k, v in r.items() if k.endswith('_gibs')})
for r in json.load(open('$OUT/make_rate.json'))['rows']: print('make', r['gib'], {k: v for k, v in r.items() if k.endswith('gibs')})"
echo done
