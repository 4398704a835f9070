#!/bin/bash
# DWT level-1 variants: kernel durations (rocprofv3 kernel trace) of single
# C2 encodes with the streaming kernel at 4- and 8-row horizontal batches
# and with the windowed kernel.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-dwtab}
mkdir -p $o
B="python bench.py --no-cpu-baseline --no-lossless --inflight 1 --steps 8 --warmup 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/rb4 -o run --output-format csv -- $B > $o/rb4.json 2> $o/rb4.err || exit 1
JP2HIP_DWT_L1_RB=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/rb8 -o run --output-format csv -- $B > $o/rb8.json 2> $o/rb8.err || exit 1
