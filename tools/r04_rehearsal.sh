#!/bin/bash
# The N > 1 DeviceShard path rehearsed on this one GPU at the default
# config-5 shard shape (32 GiB per rank, every rank on cuda:0, gloo between
# ranks: a functional run of the protocol, not a scaling measurement), with
# --check at a small shape first.  Outputs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04u}
OUT=gpurun_out/$TAG
mkdir -p $OUT
DSX_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --gib 2 --check --no-cpu > $OUT/check_n2.json 2> $OUT/check_n2.err || { tail -30 $OUT/check_n2.err; exit 1; }
echo "check n=2: $(cat $OUT/check_n2.json)"
for n in 1 2 4; do
  if [ $n = 1 ]; then
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/rehearsal_n$n.json 2> $OUT/rehearsal_n$n.err || { tail -30 $OUT/rehearsal_n$n.err; exit 1; }
  else
    DSX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 --no-cpu > $OUT/rehearsal_n$n.json 2> $OUT/rehearsal_n$n.err || { tail -30 $OUT/rehearsal_n$n.err; exit 1; }
  fi
  python3 -c "
import json;d=json.loads([l for l in open('$OUT/rehearsal_n$n.json') if l.startswith('{')][-1])
print('n=$n', d['value'], d['ms_per_step'], d['config']['parallelism'], d['config']['chunks'])"
done
echo done
