#!/bin/bash
# Tail-split default 3 vs 4 on the driver's command (3 rounds, fresh
# processes alternating), HBM read requests at the default, the 9 GiB
# two-piece parity tests, and the N > 1 DeviceShard path rehearsed on this
# one GPU (gloo between ranks, every rank on cuda:0) at the default
# config-5 shard shape.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "9gib or config5" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_configs.log 2>&1 || { tail -30 $OUT/pytest_configs.log; exit 1; }
tail -1 $OUT/pytest_configs.log
bash tools/r04_lane_ab.sh $TAG DSX_TAIL_SPLIT=3 DSX_TAIL_SPLIT=4 DSX_TAIL_SPLIT=3,DSX_TAIL_MULT=1 DSX_TAIL_SPLIT=4,DSX_TAIL_MULT=1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/pmc_rdreq -o run --output-format csv -- python3 $CMD --no-cpu > $OUT/pmc_rdreq.json 2> $OUT/pmc_rdreq.err || { tail $OUT/pmc_rdreq.err; exit 1; }
python3 tools/traffic_json.py $OUT/pmc_rdreq 8589934592 uniform > $OUT/traffic_uniform_8589934592.json && grep ratio $OUT/traffic_uniform_8589934592.json
for n in 2 4; do
  DSX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --no-cpu > $OUT/rehearsal_n$n.json 2> $OUT/rehearsal_n$n.err || { tail -30 $OUT/rehearsal_n$n.err; exit 1; }
  echo "n=$n: $(cat $OUT/rehearsal_n$n.json)"
done
echo done
