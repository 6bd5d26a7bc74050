set -o pipefail
# one-window IndexFromFile with 8 MiB read slots (DSX_INDEX_SLOT) and the
# last 32 / 64 MiB scanned per slot, against the default 32 MiB slots
mkdir -p gpurun_out/r06ad
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 12 d=12:-1 d_nomid=12:-1 d_e48=12:-1 cut > gpurun_out/r06ad/feed_s32.json 2> gpurun_out/r06ad/feed_s32.err && \
DSX_INDEX_SLOT=8388608 DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 12 d=12:-1 d_t32=12:-1 d_t64=12:-1 d_t64_e48=12:-1 d_t64_m4_e40=12:-1 cut > gpurun_out/r06ad/feed_s8.json 2> gpurun_out/r06ad/feed_s8.err
