#!/bin/bash
# Round 5 quick check: GPU suite, C3 single + 6 in flight, short C2 bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5check}
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 240 python tests/tools/c3_inflight.py 6 > $o/c3.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/bench.json 2> $o/bench.err || exit 1
