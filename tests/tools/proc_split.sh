#!/bin/bash
# Host-side check: one process x 16 images in flight vs 2 processes x 8 on the
# same GPU (gloo for the timing barrier), and 4 x 4.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-procsplit}
mkdir -p $o
timeout -k 10 200 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/p1x16.json 2> $o/p1x16.err || exit 1
JP2HIP_BENCH_DEVICE=0 JP2HIP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --inflight 8 --steps 32 --warmup 2 --no-cpu-baseline --no-lossless > $o/p2x8.json 2> $o/p2x8.err || exit 1
JP2HIP_BENCH_DEVICE=0 JP2HIP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --inflight 4 --steps 64 --warmup 2 --no-cpu-baseline --no-lossless > $o/p4x4.json 2> $o/p4x4.err || exit 1
for f in p1x16 p2x8 p4x4; do python -c "import json; d=json.loads(open('$o/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['n_gpus'])"; done | tee $o/summary.txt
