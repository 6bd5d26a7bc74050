set -o pipefail
# the contexts' streams at the highest priority against the default (the
# headline bench line, alternating processes, diagnostic build both); then
# VerifyIndex / IndexFromFile shares A/B at 1 GiB
mkdir -p gpurun_out/r06ak
export TMPDIR=/tmp
timeout -k 10 600 python tools/ab.py gpurun_out/r06ak/prio hi:diag def:diag,DSX_CTX_PRIO=0 --rounds 4 > gpurun_out/r06ak/prio.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 d=12:-1 d_nomid=12:-1 v=12:-1 v_nomid=12:-1 cut > gpurun_out/r06ak/feed_1g.json 2> gpurun_out/r06ak/feed_1g.err
