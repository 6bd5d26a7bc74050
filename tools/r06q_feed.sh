set -o pipefail
mkdir -p gpurun_out/r06q
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06q/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d12=12:-1 d12_nomid=12:-1 d12_mid4=12:-1 d12_mid6=12:-1 v12=12:-1 cut > gpurun_out/r06q/feed_ab.json 2> gpurun_out/r06q/feed_ab.err
