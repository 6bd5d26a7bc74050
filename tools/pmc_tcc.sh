#!/bin/bash
# L2 memory-side request sizes and hit rates of the scan (4 GiB, beyond the
# 256 MiB Infinity Cache); one rocprofv3 --pmc pass per counter group.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tcc}
G=${GIB:-4}
mkdir -p $OUT
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python bench.py --gib $G --steps 5 --warmup 1 --no-cpu > $OUT/p$i.log 2>&1 || exit 1
  python tools/pmc_summary.py $OUT/p$i
done
