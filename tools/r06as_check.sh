set -o pipefail
# after the geometry / cut helpers refactor: the GPU suite, smoke, bench and
# the one-window A/B
mkdir -p gpurun_out/r06as
export TMPDIR=/tmp
O=gpurun_out/r06as
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 d=12:-1 v=12:-1 cut > $O/feed_1g.json 2> $O/feed_1g.err
