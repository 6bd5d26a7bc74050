#!/bin/bash
# Scan ablations (DSX_SCAN_VARIANT: 0 full, 1 no boundary test, 3 staging only,
# 4 no staging) at 1 and 4 GiB, then SQ/GRBM counters of the full scan.
set -o pipefail
# ablation variants are in the diagnostic build (make -C desync_amd/csrc diag)
export DSX_LIB_PATH=$PWD/desync_amd/libdsx_diag.so
export TMPDIR=/tmp
OUT=gpurun_out/${1:-abl}
mkdir -p $OUT
for g in 1 4; do
for v in 0 1 3 4; do
  for w in uniform zeros; do
  r=$(DSX_SCAN_VARIANT=$v timeout -k 10 120 python bench.py --gib $g --workload $w --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "gib=$g variant=$v $w $r"
  done
done
done | tee $OUT/ablate.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc1 -o run --output-format csv -- python bench.py --gib 4 --steps 5 --warmup 1 --no-cpu > $OUT/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d $OUT/pmc2 -o run --output-format csv -- python bench.py --gib 4 --steps 5 --warmup 1 --no-cpu > $OUT/pmc2.log 2>&1 || exit 1
python tools/pmc_summary.py $OUT/pmc1
python tools/pmc_summary.py $OUT/pmc2
