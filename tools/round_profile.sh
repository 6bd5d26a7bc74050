#!/bin/bash
# Round measurement on the GPU box: full GPU parity suite, the bench line,
# rocprofv3 kernel-trace stats and a FETCH_SIZE pass, the host-resident rate
# and the other workloads.  Outputs under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1100 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/pmc_bench.json 2> $OUT/pmc.err || { tail $OUT/pmc.err; exit 1; }
timeout -k 10 300 python tools/host_rate.py 1 > $OUT/host_rate.json 2> $OUT/host_rate.err || { tail $OUT/host_rate.err; exit 1; }
cat $OUT/host_rate.json
for w in dedup zeros; do
  timeout -k 10 300 python bench.py --workload $w --gib 4 --no-cpu > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail $OUT/bench_$w.err; exit 1; }
  cat $OUT/bench_$w.json
done
