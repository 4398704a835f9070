#!/bin/bash
# MQ modeller scheduled with the interval chain ahead of the table wait
# (JP2HIP_MQ_SCHED=1, the product) vs without: parity, census (debug builds),
# single-image stage times, C2 bench A/B, C3 in flight.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5sched}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/parity.txt 2>&1 || exit 1
for D in libjp2hip_debug libjp2hip_dbgsched0; do
  JP2HIP_LIBRARY=$L/$D.so timeout -k 10 200 python tests/tools/mq_census.py > $o/census_$D.txt 2>&1 || exit 1
done
for P in libjp2hip libjp2hip_sched0; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
bash tests/tools/ab_lib.sh $(basename $o)/ab $L/libjp2hip.so $L/libjp2hip_sched0.so 2 || exit 1
for P in libjp2hip libjp2hip_sched0; do
  JP2HIP_LIBRARY=$L/$P.so C3_EACH=4 timeout -k 10 300 python tests/tools/c3_inflight.py 8 > $o/c3_$P.json 2> $o/c3_$P.err || exit 1
done
