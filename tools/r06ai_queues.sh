#!/bin/bash
# Queue acquisition: at stream creation or at first use?  (idle streams
# created first and never used); our streams at the highest priority beside
# a torch-like pool of 32 default-priority streams.
set -e
mkdir -p gpurun_out/r06ai
o=gpurun_out/r06ai/queues.jsonl
: > $o
timeout -k 10 30 ./tools/queue_probe 3 1 0 0 >> $o
timeout -k 10 30 ./tools/queue_probe 3 1 0 4 >> $o
timeout -k 10 30 ./tools/queue_probe 3 1 0 32 >> $o
timeout -k 10 30 ./tools/queue_probe 4 1 3 32 >> $o
timeout -k 10 30 ./tools/queue_probe 5 1 3 0 >> $o
