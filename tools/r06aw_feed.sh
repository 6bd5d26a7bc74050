set -o pipefail
# one more box: one-window IndexFromFile / VerifyIndex at 1 GiB on the final
# defaults, 20 in-process rounds
mkdir -p gpurun_out/r06aw
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 20 d=12:-1 v=12:-1 cut > gpurun_out/r06aw/feed_1g.json 2> gpurun_out/r06aw/feed_1g.err
