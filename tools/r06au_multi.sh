set -o pipefail
# VerifyIndex: shares in the last of several windows (DSX_SHARE_MULTI A/B)
# the index tests, then the N > 1 rehearsal (ranks sharing the GPU over gloo)
mkdir -p gpurun_out/r06au
export TMPDIR=/tmp
O=gpurun_out/r06au
timeout -k 10 500 python -u -m pytest tests/test_gpu_index.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py --gib=2 10 d=12:-1 v=12:-1 v_u0=12:-1 cut > $O/feed_2g.json 2> $O/feed_2g.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py --gib=4 6 d=12:-1 v=12:-1 v_u0=12:-1 cut > $O/feed_4g.json 2> $O/feed_4g.err && \
true
