set -o pipefail
# one-window IndexFromFile: GPU shares (digest_kernel on the side streams)
# and the end digest on digest_pc_kernel; end cuts 64 / 48 / 40 / 32 KiB
mkdir -p gpurun_out/r06ab
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06ab/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_nomid=12:-1 d_m4_e48=12:-1 d_m4_e40=12:-1 d_m4_e32=12:-1 v12=12:-1 cut > gpurun_out/r06ab/feed_ab.json 2> gpurun_out/r06ab/feed_ab.err
