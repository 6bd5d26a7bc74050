set -o pipefail
# one-window IndexFromFile: two shares whatever the end cut (the points
# follow the feeder's cut), end cuts 48 / 44 / 40 KiB
mkdir -p gpurun_out/r06aq
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_e44=12:-1 d_e40=12:-1 d_e36=12:-1 cut > gpurun_out/r06aq/feed_1g.json 2> gpurun_out/r06aq/feed_1g.err
