#!/bin/bash
# Lossless C3, 6 contexts in flight, alternating libraries.
set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
o=gpurun_out/${1:-c3ab}; shift
mkdir -p $o
for r in 1 2; do
for t in "$@"; do
  echo "$t $r $(JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/$t.so C3_EACH=6 timeout -k 10 200 python tests/tools/c3_inflight.py 6 2> $o/$t.err | tail -1)" >> $o/summary.txt || exit 1
done
done
