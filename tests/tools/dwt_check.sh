#!/bin/bash
# DWT change check: the parity tests that exercise the DWT (every codestream
# case, C2/C3 full size, tiled/compressed inputs), then a kernel trace of
# single-image C2 encodes (DWT kernel durations alone).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-dwtc}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_split.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --batch 1 --steps 8 --warmup 1 > $o/kt.json 2> $o/kt.err || exit 1
