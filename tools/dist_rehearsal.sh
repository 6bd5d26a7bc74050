#!/bin/bash
# N>1 bench path rehearsed on a one-GPU box: 2 and 3 ranks share the GPU,
# gloo for the collectives, --check compares the concatenated per-rank cut
# lists with one dsx_cut_device over the whole blob.
set -o pipefail
for n in 2 3; do
  DSX_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --gib ${GIB:-0.25} \
    --check --steps 3 --warmup 1 --no-cpu > gpurun_out/dist_$n.json 2> gpurun_out/dist_$n.err || { tail -20 gpurun_out/dist_$n.err; exit 1; }
  grep -h "check ok" gpurun_out/dist_$n.err
  grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*' gpurun_out/dist_$n.json | tr '\n' ' '; echo
done
