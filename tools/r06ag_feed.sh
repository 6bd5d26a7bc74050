set -o pipefail
# one-window IndexFromFile, streaming feeder: four shares with slack (the
# shares may end after the read) at 45 ns/B and lower end cuts
mkdir -p gpurun_out/r06ag
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so DSX_TAIL_LOG=1 timeout -k 10 400 python tools/feed_ab.py 14 d=12:-1 d_e48=12:-1 d_n45_s1500_e36=12:-1 d_n45_s1500_e48=12:-1 d_n45_s1000_e32=12:-1 d_s1500_e40=12:-1 cut > gpurun_out/r06ag/feed_ab.json 2> gpurun_out/r06ag/feed_ab.err
