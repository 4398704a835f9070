#!/bin/bash
# MQ census experiments (debug builds): product chains, the modeller alone,
# the modeller alone without its next-state LDS read.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5mqexp}
mkdir -p $o
for L in libjp2hip_debug libjp2hip_mqexp2 libjp2hip_mqexp3; do
  JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/$L.so timeout -k 10 200 python tests/tools/mq_census.py > $o/$L.txt 2>&1 || exit 1
done
