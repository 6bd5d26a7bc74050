set -o pipefail
# one-window IndexFromFile: the shares' cuts at the chain rate they showed in
# the trace (37-40 ns/B, profiles/r06an) instead of 58, at most two shares
mkdir -p gpurun_out/r06ao
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_n40_m2=12:-1 d_n45_m2=12:-1 d_n40_m2_e40=12:-1 d_n45_m3=12:-1 cut > gpurun_out/r06ao/feed_ab.json 2> gpurun_out/r06ao/feed_ab.err
