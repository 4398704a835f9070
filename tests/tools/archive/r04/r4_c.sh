#!/bin/bash
# Deflate window decoder on the GPU: the compressed-strip / inflate tests and
# the split tests with Deflate masters, then the ingest cost per codec.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4c}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_split.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "deflate or compressed or inflate or tiled" > $o/t.log 2>&1 || exit 1
timeout -k 10 300 python tests/tools/ingest_codecs.py --rps 64 --reps 3 > $o/ingest.jsonl 2> $o/ingest.err || exit 1
