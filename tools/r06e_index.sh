set -o pipefail
mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06e/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 d12=12:-1 d12_nomid=12:-1 c40=12:40960 c48=12:49152 t28_nomid=28:28672 v12=12:-1 cut > gpurun_out/r06e/feed_ab.json 2> gpurun_out/r06e/feed_ab.err && \
timeout -k 10 400 python tools/window_dip.py 8 1 2 4 > gpurun_out/r06e/window_dip.json 2> gpurun_out/r06e/window_dip.err
