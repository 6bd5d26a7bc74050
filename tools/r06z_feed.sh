set -o pipefail
# GPU shares of a one-window IndexFromFile call at several points during the
# read (side streams on their own queues): schedules and end cuts
mkdir -p gpurun_out/r06z
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06z/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 12 d=12:-1 d_nomid=12:-1 d_m1=12:-1 d_m2_e48=12:-1 d_m3_e32=12:-1 d_m3_e24=12:-1 v12=12:-1 cut > gpurun_out/r06z/feed_ab.json 2> gpurun_out/r06z/feed_ab.err
