set -o pipefail
# the final code: GPU suite, smoke, bench; IndexFromFile / VerifyIndex A/B at
# 1 / 2 / 4 GiB (VerifyIndex's shares in the last of several windows against
# none, DSX_SHARE_MULTI=0), make_rate
mkdir -p gpurun_out/r06av
export TMPDIR=/tmp
O=gpurun_out/r06av
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 d=12:-1 v=12:-1 cut > $O/feed_1g.json 2> $O/feed_1g.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py --gib=2 10 d=12:-1 d_u0=12:-1 v=12:-1 v_u0=12:-1 cut > $O/feed_2g.json 2> $O/feed_2g.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py --gib=4 6 d=12:-1 d_u0=12:-1 v=12:-1 v_u0=12:-1 cut > $O/feed_4g.json 2> $O/feed_4g.err && \
timeout -k 10 600 python tools/make_rate.py 1 2 4 > $O/make_rate.json 2> $O/make_rate.err
