#!/bin/bash
# Hardware-queue sharing among streams (tools/queue_probe.hip), box defaults
# and with more queues allowed.
set -e
mkdir -p gpurun_out/r06w
o=gpurun_out/r06w/queues.jsonl
: > $o
for n in 3 4 5 6; do
  timeout -k 10 30 ./tools/queue_probe $n 1 >> $o
done
timeout -k 10 30 ./tools/queue_probe 5 0 >> $o
GPU_MAX_HW_QUEUES=8 timeout -k 10 30 ./tools/queue_probe 5 1 >> $o
GPU_MAX_HW_QUEUES=8 timeout -k 10 30 ./tools/queue_probe 6 1 >> $o
timeout -k 10 30 ./tools/queue_probe 5 1 1 >> $o
timeout -k 10 30 ./tools/queue_probe 6 1 2 >> $o
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}" >> $o
# the one-window IndexFromFile call at the box's queue count and at 8
export TMPDIR=/tmp
DSX_LIB_PATH=desync_amd/libdsx_diag.so timeout -k 10 200 python tools/feed_ab.py 10 d=12:-1 v=12:-1 cut > gpurun_out/r06w/feed_q4.json 2> gpurun_out/r06w/feed_q4.err
GPU_MAX_HW_QUEUES=8 DSX_LIB_PATH=desync_amd/libdsx_diag.so timeout -k 10 200 python tools/feed_ab.py 10 d=12:-1 v=12:-1 cut > gpurun_out/r06w/feed_q8.json 2> gpurun_out/r06w/feed_q8.err
