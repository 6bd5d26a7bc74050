set -o pipefail
# the streaming tail feeder (a group queue the host pool drains while batches
# arrive): one-window IndexFromFile at end cuts 64 / 48 / 40 KiB
mkdir -p gpurun_out/r06af
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r06af/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_e48=12:-1 d_e40=12:-1 d_m4_e40=12:-1 d_t0=12:-1 v12=12:-1 cut > gpurun_out/r06af/feed_ab.json 2> gpurun_out/r06af/feed_ab.err
