set -o pipefail
# the two-cut GPU share of a one-window IndexFromFile call with the side
# streams at the lowest priority (their own HSA queues) against the default
# priority (sharing one with the pipeline's streams, tools/queue_probe)
mkdir -p gpurun_out/r06x
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06x/pytest_index.txt 2>&1 && \
DSX_SIDE_PRIO=1 DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 12 d12=12:-1 d12_nomid=12:-1 d12_mid3=12:-1 d12_mid7=12:-1 v12=12:-1 cut > gpurun_out/r06x/feed_low.json 2> gpurun_out/r06x/feed_low.err && \
DSX_SIDE_PRIO=0 DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 12 d12=12:-1 d12_nomid=12:-1 d12_mid3=12:-1 d12_mid7=12:-1 v12=12:-1 cut > gpurun_out/r06x/feed_def.json 2> gpurun_out/r06x/feed_def.err
