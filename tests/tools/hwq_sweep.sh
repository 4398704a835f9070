#!/bin/bash
# C2 bench line at several hardware-queue counts per process.
set -o pipefail
o=gpurun_out/${1:-hwq}
mkdir -p $o
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline --no-lossless --steps 48 > $o/q$q.json 2> $o/q$q.err || exit 1
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python bench.py --no-cpu-baseline --no-lossless --steps 48 --inflight 16 > $o/q16i16.json 2> $o/q16i16.err || exit 1
