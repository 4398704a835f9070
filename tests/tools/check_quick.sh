#!/bin/bash
# Quick GPU check: the parity suite, a short C2 bench, and a rocprofv3 kernel
# trace of single-image encodes.
#   tests/tools/check_quick.sh <out-name>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-q}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-lossless > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --batch 1 --steps 12 --warmup 2 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-lossless > $o/bench_rocprof.json 2> $o/bench_rocprof.err || exit 1
