#!/bin/bash
# The warm-up handoff with DSX_TAIL_SPLIT = 4 as the default: the GPU suite,
# then the driver's command against libdsx_base.so (no handoff, k = 3) in
# alternating fresh processes, and the new scan's L2 read requests.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
BASE=$PWD/desync_amd/libdsx_base.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for i in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then L="DSX_LIB_PATH=$BASE"; else L="DSX_SCAN_HANDOFF=1"; fi
    env $L timeout -k 10 200 python3 $CMD > $OUT/c5_${lib}_$i.json 2> $OUT/c5_${lib}_$i.err || { tail $OUT/c5_${lib}_$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/c5_${lib}_$i.json'));r=d['roofline']
print('config5 $lib #$i', d['value'], d['ms_per_step'], r['kernel_ms'], r['clock_mhz'], r.get('wave_busy'), r['scan_share_of_step'])"
  done
done
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/pmc_rdreq -o run --output-format csv -- python3 $CMD > $OUT/pmc_rdreq.json 2> $OUT/pmc_rdreq.err || { tail $OUT/pmc_rdreq.err; exit 1; }
python3 tools/traffic_json.py $OUT/pmc_rdreq 8589934592 uniform > $OUT/traffic_uniform_8589934592.json && grep ratio $OUT/traffic_uniform_8589934592.json
echo done
