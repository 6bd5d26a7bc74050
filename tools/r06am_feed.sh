set -o pipefail
# one-window IndexFromFile: the readers' 4 CPUs join the feeder's hashers
# once the reads are done (DSX_FEED_EXTRA), at end cuts 48 / 40 KiB
mkdir -p gpurun_out/r06am
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r06am/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_x0=12:-1 d_e40=12:-1 d_e40_x0=12:-1 d_e32=12:-1 cut > gpurun_out/r06am/feed_ab.json 2> gpurun_out/r06am/feed_ab.err
