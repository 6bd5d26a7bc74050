#!/bin/bash
# N>1 bench path rehearsed on a one-GPU box: ranks share the GPU, gloo for
# the collectives (RCCL needs one GPU per rank).  Small shards with --check
# (the concatenated per-rank cut lists against one dsx_cut_device over the
# whole blob), then N = 2 at the full 32 GiB shard shape.  Prints what the
# line reports about itself: dist backend / world size, every rank's scan
# roofline, every rank's HBM footprint.
#   tools/dist_rehearsal.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/dist}
mkdir -p $OUT
run() {  # n gib extra-args...
  local n=$1 gib=$2; shift 2
  DSX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --gib $gib \
    --no-cpu "$@" > $OUT/dist_${n}_${gib}.json 2> $OUT/dist_${n}_${gib}.err || { tail -20 $OUT/dist_${n}_${gib}.err; exit 1; }
  grep -h "check ok" $OUT/dist_${n}_${gib}.err
  python3 - $OUT/dist_${n}_${gib}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r, h = d["roofline"], d["hbm"]
print(f"N={d['n_gpus']} value={d['value']} GiB/s dist={d['dist']} frac_min={r['frac']} "
      f"per_rank={[(x['frac'], x['kernel_ms'], x['launches']) for x in r['per_rank']]} "
      f"hbm_per_rank_GiB={[round(b / 2**30, 2) for b in h['per_rank_bytes']]} "
      f"contexts_MiB={[round(b / 2**20, 1) for b in h['rank0']['context_bytes']]} max_frac={h['max_frac']}")
PY
}
run 2 0.25 --check --steps 3 --warmup 1
run 3 0.25 --check --steps 3 --warmup 1
run 2 32 --steps 10 --warmup 3
