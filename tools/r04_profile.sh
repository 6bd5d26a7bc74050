#!/bin/bash
# Round-4 measurement of the driver's exact command and the cold regime:
#   1. the GPU suite;
#   2. the driver's bench command (config-5 shard default) with board power
#      sampled, then the same command under rocprofv3 --kernel-trace --stats,
#      an L2 read-request --pmc pass (HBM bytes per launch) and a
#      GRBM_GUI_ACTIVE / SQ_BUSY_CYCLES pass (clock per dispatch);
#   3. config 2's 1 GiB shape under the same protocol, DSX_FUSE 0/1 in
#      alternating fresh processes (both on libdsx_diag.so, which holds the
#      fused stitch);
#   4. per-launch in-kernel stamps from idle and after a 1 s gap;
#   5. energy per GiB of the staging alternatives (tools/ubench_energy.hip).
# Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 tools/power_sample.sh $OUT/power_bench.txt -- python3 $CMD > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 tools/power_summary.py $OUT/power_bench.txt > $OUT/power_bench.json && cat $OUT/power_bench.json
# the stamps' own cost: the same command without them, and once more with
DSX_BENCH_STAMPS=0 timeout -k 10 200 python3 $CMD --no-cpu > $OUT/bench_nostamps.json 2> $OUT/bench_nostamps.err || { tail $OUT/bench_nostamps.err; exit 1; }
timeout -k 10 200 python3 $CMD --no-cpu > $OUT/bench_2.json 2> $OUT/bench_2.err || { tail $OUT/bench_2.err; exit 1; }
echo "no stamps: $(cat $OUT/bench_nostamps.json)"; echo "again: $(cat $OUT/bench_2.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $CMD > $OUT/trace_bench.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
cat $OUT/trace_bench.json
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/pmc_rdreq -o run --output-format csv -- python3 $CMD --no-cpu > $OUT/pmc_rdreq.json 2> $OUT/pmc_rdreq.err || { tail $OUT/pmc_rdreq.err; exit 1; }
python3 tools/traffic_json.py $OUT/pmc_rdreq 8589934592 uniform > $OUT/traffic_uniform_8589934592.json && cat $OUT/traffic_uniform_8589934592.json
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $OUT/pmc_clk -o run --output-format csv -- python3 $CMD --no-cpu > $OUT/pmc_clk.json 2> $OUT/pmc_clk.err || { tail $OUT/pmc_clk.err; exit 1; }
for i in 1 2; do
  for f in 0 1; do
    DSX_LIB_PATH=$PWD/desync_amd/libdsx_diag.so DSX_FUSE=$f timeout -k 10 120 python3 $CMD --config2 --no-cpu > $OUT/c2_fuse${f}_$i.json 2> $OUT/c2_fuse${f}_$i.err || { tail $OUT/c2_fuse${f}_$i.err; exit 1; }
    echo "fuse=$f #$i $(cat $OUT/c2_fuse${f}_$i.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_c2 -o run --output-format csv -- python3 $CMD --config2 --no-cpu > $OUT/trace_c2.json 2> $OUT/trace_c2.err || { tail $OUT/trace_c2.err; exit 1; }
timeout -k 10 200 python3 tools/cold_regime.py --gib 1 --jobs 60 --out $OUT/cold_1g.json > $OUT/cold_1g.txt 2> $OUT/cold_1g.err || { tail $OUT/cold_1g.err; exit 1; }
timeout -k 10 200 python3 tools/cold_regime.py --gib 32 --seed 3 --jobs 12 --out $OUT/cold_32g.json > $OUT/cold_32g.txt 2> $OUT/cold_32g.err || { tail $OUT/cold_32g.err; exit 1; }
head -30 $OUT/cold_1g.txt
if [ -x tools/ubench_energy ]; then
  timeout -k 10 180 ./tools/ubench_energy 8 1.5 > $OUT/ubench_energy.txt 2>&1 || { tail $OUT/ubench_energy.txt; exit 1; }
  cat $OUT/ubench_energy.txt
fi
echo done
