set -o pipefail
mkdir -p gpurun_out/r06n
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 16 c64=12:65536 c64_noslot=12:65536 c56=12:57344 c56_noslot=12:57344 c80=12:81920 c80_noslot=12:81920 cut > gpurun_out/r06n/feed_ab.json 2> gpurun_out/r06n/feed_ab.err
