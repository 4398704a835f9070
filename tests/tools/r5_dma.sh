#!/bin/bash
# Round 5: code-stream D2H on SDMA (product) against the blit build: GPU
# suite, then C2 bench and C3 lossless A/B, alternating.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5dma}
mkdir -p $o
timeout -k 10 120 tests/tools/probe/sdma_copy_probe > $o/probe.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
bash tests/tools/ab_lib.sh $(basename $o)/ab jp2-bucketeer_amd/jp2hip/libjp2hip.so jp2-bucketeer_amd/jp2hip/libjp2hip_blit.so 2 || exit 1
for L in libjp2hip libjp2hip_blit libjp2hip libjp2hip_blit; do
  JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/$L.so timeout -k 10 240 python tests/tools/c3_inflight.py 6 > $o/c3_$L.txt 2>&1 || exit 1
  echo "$L $(tail -1 $o/c3_$L.txt)" >> $o/c3_summary.txt
done
