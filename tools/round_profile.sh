#!/bin/bash
# Round measurement on the GPU box: GPU parity suite, the bench line (with
# board power / clock sampled while it runs), a rocprofv3 kernel-trace/stats
# pass and an L2 memory-request pass of the same command, the host-resident
# rate and the other workloads.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 tools/power_sample.sh $OUT/power_bench.txt -- python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python tools/power_summary.py $OUT/power_bench.txt > $OUT/power_bench.json && cat $OUT/power_bench.json
# the same command under the kernel trace (steady state: 100 warm-up jobs)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --no-cpu > $OUT/trace_bench.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/pmc_rdreq -o run --output-format csv -- python bench.py --no-cpu --steps 10 --warmup 2 > $OUT/pmc_bench.json 2> $OUT/pmc.err || { tail $OUT/pmc.err; exit 1; }
python tools/traffic_json.py $OUT/pmc_rdreq 1073741824 uniform > $OUT/traffic_uniform.json
cat $OUT/traffic_uniform.json
timeout -k 10 300 python tools/host_rate.py 1 > $OUT/host_rate.json 2> $OUT/host_rate.err || { tail $OUT/host_rate.err; exit 1; }
cat $OUT/host_rate.json
for w in dedup zeros; do
  timeout -k 10 300 python bench.py --workload $w --gib 4 --no-cpu --warmup 30 --steps 100 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail $OUT/bench_$w.err; exit 1; }
  cat $OUT/bench_$w.json
done
timeout -k 10 300 python tools/digest_rate.py 1 4 16 > $OUT/digest_rate.json 2> $OUT/digest_rate.err || { tail $OUT/digest_rate.err; exit 1; }
cat $OUT/digest_rate.json
timeout -k 10 300 python tools/make_rate.py > $OUT/make_rate.json 2> $OUT/make_rate.err || { tail $OUT/make_rate.err; exit 1; }
cat $OUT/make_rate.json
timeout -k 10 300 python tools/stream_rate.py > $OUT/stream_rate.json 2> $OUT/stream_rate.err || { tail $OUT/stream_rate.err; exit 1; }
cat $OUT/stream_rate.json
