set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/p1 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu --inflight 1 > gpurun_out/pmc/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d gpurun_out/pmc/p2 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu --inflight 1 > gpurun_out/pmc/p2.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/pmc/p1
python tools/pmc_summary.py gpurun_out/pmc/p2
