set -o pipefail
mkdir -p gpurun_out/r06l
export TMPDIR=/tmp
grep -m1 "model name" /proc/cpuinfo > gpurun_out/r06l/cpu.txt; grep -m1 flags /proc/cpuinfo | tr ' ' '\n' | grep -E "sha|avx512|vaes|gfni" | tr '\n' ' ' >> gpurun_out/r06l/cpu.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06l/pytest_index.txt 2>&1 && \
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 c48=12:49152 c64=12:65536 c40=12:40960 v12=12:-1 cut > gpurun_out/r06l/feed_ab.json 2> gpurun_out/r06l/feed_ab.err
