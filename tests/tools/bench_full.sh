#!/bin/bash
# The driver's bench command (default flags and the round-end flags).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-bf}
mkdir -p $o
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench_driver.json 2> $o/bench_driver.err || exit 1
