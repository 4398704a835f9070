#!/bin/bash
# k_t1_mq residency sensitivity: the product against builds whose MQ
# workgroups hold more LDS (7 and 5 per CU instead of 8): C3 in flight (8
# contexts, twice) and the C2 bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5lds}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
for r in 1 2; do
  for V in libjp2hip libjp2hip_lds7 libjp2hip_lds5; do
    JP2HIP_LIBRARY=$L/$V.so C3_EACH=4 timeout -k 10 300 python tests/tools/c3_inflight.py 8 > $o/c3_${V}_$r.json 2> $o/c3_${V}_$r.err || exit 1
    echo "$V $r $(grep inflight $o/c3_${V}_$r.json)" | tee -a $o/summary.txt
  done
done
bash tests/tools/ab_lib.sh $(basename $o)/ab $L/libjp2hip.so $L/libjp2hip_lds5.so 2 || exit 1
