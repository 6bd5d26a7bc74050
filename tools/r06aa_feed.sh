set -o pipefail
# the index path's digests on digest_pc_kernel (DSX_DIGEST_PC=1) against the
# automatic choice (digest_kernel: the windows' chunk bound len/min is above
# the pc kernel's 32 K), one-window IndexFromFile with and without GPU shares
mkdir -p gpurun_out/r06aa
export TMPDIR=/tmp
DSX_DIGEST_PC=1 DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 10 d=12:-1 d_nomid=12:-1 d_m3_e32=12:-1 d_m3_e24=12:-1 cut > gpurun_out/r06aa/feed_pc.json 2> gpurun_out/r06aa/feed_pc.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 10 d=12:-1 d_nomid=12:-1 d_m3_e32=12:-1 d_m3_e24=12:-1 cut > gpurun_out/r06aa/feed_auto.json 2> gpurun_out/r06aa/feed_auto.err
