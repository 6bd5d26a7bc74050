set -o pipefail
# the final defaults (shares at 45 ns/B, at most two at 1 GiB, the readers'
# CPUs joining the feeder): index tests, then 1 / 2 GiB in-process A/B
mkdir -p gpurun_out/r06ap
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r06ap/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_n58=12:-1 d_nomid=12:-1 v=12:-1 cut > gpurun_out/r06ap/feed_1g.json 2> gpurun_out/r06ap/feed_1g.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so timeout -k 10 300 python tools/feed_ab.py --gib=2 8 d=12:-1 v=12:-1 cut > gpurun_out/r06ap/feed_2g.json 2> gpurun_out/r06ap/feed_2g.err
