set -o pipefail
# kernel trace of one-window IndexFromFile and VerifyIndex calls (1 GiB): the
# GPU's shares beside the read's scans
mkdir -p gpurun_out/r06an
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r06an/trace -o run --output-format csv -- python3 tools/index_trace.py 1 --verify > gpurun_out/r06an/run.txt 2>&1 && \
python3 tools/index_trace.py --summary gpurun_out/r06an/trace > gpurun_out/r06an/summary.txt 2>&1
