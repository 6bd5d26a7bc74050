set -o pipefail
# one-window IndexFromFile: the shares on digest_pc_kernel; their cut model
# (58 / 45 ns per byte) and the end cut
mkdir -p gpurun_out/r06ac
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_nomid=12:-1 d_k0=12:-1 d_m4_e48=12:-1 d_m4_e40=12:-1 d_n45_m4_e48=12:-1 d_n45_m4_e40=12:-1 cut > gpurun_out/r06ac/feed_ab.json 2> gpurun_out/r06ac/feed_ab.err
