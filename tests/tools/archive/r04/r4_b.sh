#!/bin/bash
# round 4 pass b: the Deflate rework on the GPU (compressed-strip tests, the
# crafted every-distance stream, ingest cost), then MQ issue-priority A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4b}
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "deflate or compressed or inflate or tiled" > $o/t.log 2>&1 || exit 1
timeout -k 10 300 python tests/tools/ingest_codecs.py --rps 64 --reps 3 > $o/ingest.jsonl 2> $o/ingest.err || exit 1
L=jp2-bucketeer_amd/jp2hip
bash tests/tools/ab_kt.sh ${1:-r4b}/ab_prio $L/libjp2hip.so $L/libjp2hip_prio1.so $L/libjp2hip_prio3.so || exit 1
