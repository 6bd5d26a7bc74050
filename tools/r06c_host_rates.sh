set -o pipefail
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
nproc > gpurun_out/r06c/nproc.txt; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS" >> gpurun_out/r06c/nproc.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r06c/nproc.txt 2>&1 || true
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 300 python tools/feed_ab.py 14 d12=12:-1 c48=12:49152 c96=12:98304 t28=28:28672 v12=12:-1 cut > gpurun_out/r06c/feed_ab.json 2> gpurun_out/r06c/feed_ab.err && \
timeout -k 10 400 python tools/window_dip.py 8 1 2 4 > gpurun_out/r06c/window_dip.json 2> gpurun_out/r06c/window_dip.err
