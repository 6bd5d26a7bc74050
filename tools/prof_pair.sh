set -o pipefail
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
G2="GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES"
DSX_SCAN_VARIANT=4 STEPS=4 bash tools/profile_scan.sh p5v4 "$G1" "$G2" && python tools/pmc_summary.py gpurun_out/p5v4 > gpurun_out/p5v4/summary.txt && STEPS=4 bash tools/profile_scan.sh p5v0 "$G1" "$G2" && python tools/pmc_summary.py gpurun_out/p5v0 > gpurun_out/p5v0/summary.txt
