set -o pipefail
mkdir -p gpurun_out/r06f
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 c40=12:40960 c48=12:49152 c64=12:65536 c80=12:81920 r3c56=13:57344:3 c64_mid=12:65536 v12=12:-1 cut > gpurun_out/r06f/feed_ab.json 2> gpurun_out/r06f/feed_ab.err
