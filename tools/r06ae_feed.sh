set -o pipefail
# one-window IndexFromFile: the call's last 32 / 64 MiB in 8 / 4 MiB pieces
mkdir -p gpurun_out/r06ae
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r06ae/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_t0=12:-1 d_t64=12:-1 d_t32_d8=12:-1 d_e48=12:-1 d_t64_e48=12:-1 cut > gpurun_out/r06ae/feed_ab.json 2> gpurun_out/r06ae/feed_ab.err
