set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p1
for cv in 0:0 0:1 0:3 0:4 1:0 1:1 1:4 2:0; do
  c=${cv%:*}; v=${cv#*:}
  r=$(DSX_SCAN_CFG=$c DSX_SCAN_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "cfg=$c variant=$v $r"
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/p1/pmc1 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/p1/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d gpurun_out/p1/pmc2 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/p1/pmc2.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/p1/pmc1
python tools/pmc_summary.py gpurun_out/p1/pmc2
