#!/bin/bash
# Kernel trace of the C2 bench under its default load (12 images in flight):
# which kernels overlap, and for how long each runs alone.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-tl}
mkdir -p $o
python -c "import os; print('GPU_MAX_HW_QUEUES', os.environ.get('GPU_MAX_HW_QUEUES'))" > $o/env.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/kt -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --steps 48 > $o/bench.json 2> $o/bench.err || exit 1
