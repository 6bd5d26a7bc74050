set -o pipefail
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06d/pytest_index.txt 2>&1 && \
timeout -k 10 400 python tools/window_dip.py 8 1 2 4 > gpurun_out/r06d/window_dip.json 2> gpurun_out/r06d/window_dip.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py --gib=2 10 d12=12:-1 t28=28:28672 v12=12:-1 cut > gpurun_out/r06d/feed_ab_2g.json 2> gpurun_out/r06d/feed_ab_2g.err
