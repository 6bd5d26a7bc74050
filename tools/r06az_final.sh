set -o pipefail
# the round's final code: GPU suite, smoke, the default bench line
mkdir -p gpurun_out/r06az
export TMPDIR=/tmp
O=gpurun_out/r06az
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
