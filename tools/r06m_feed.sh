set -o pipefail
mkdir -p gpurun_out/r06m
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06m/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 c48=12:49152 c64=12:65536 c40=12:40960 c32=12:32768 v12=12:-1 cut > gpurun_out/r06m/feed_ab.json 2> gpurun_out/r06m/feed_ab.err && \
timeout -k 10 400 python tools/window_dip.py 8 1 2 4 > gpurun_out/r06m/window_dip.json 2> gpurun_out/r06m/window_dip.err
