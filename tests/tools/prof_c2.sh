#!/bin/bash
# C2 bench lines (12 in flight and 1 in flight) and a rocprofv3 kernel trace
# of the single-image chain.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-prof}
mkdir -p $o
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 48 > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-lossless --inflight 1 --steps 16 > $o/bench_if1.json 2> $o/bench_if1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --steps 16 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
