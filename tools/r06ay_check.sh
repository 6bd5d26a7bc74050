set -o pipefail
# the measured host rate in VerifyIndex's budget: index tests, 1 / 2 GiB A/B
mkdir -p gpurun_out/r06ay
export TMPDIR=/tmp
O=gpurun_out/r06ay
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 d=12:-1 v=12:-1 cut > $O/feed_1g.json 2> $O/feed_1g.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py --gib=2 8 v=12:-1 cut > $O/feed_2g.json 2> $O/feed_2g.err
