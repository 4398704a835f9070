#!/bin/bash
# k_t1_mq alone (HIP events, one image at a time), alternating libraries.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-mqalone}; shift
mkdir -p $o
for r in 1 2; do
for t in "$@"; do
  JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/$t.so timeout -k 10 200 python tests/tools/mq_alone.py >> $o/summary.txt 2> $o/$t.err || exit 1
done
done
