#!/bin/bash
# Masked MQ modeller A/B: parity, census (debug builds), the single-image
# stage times and the C2 bench against the compare/select formulation.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5masks}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/parity.txt 2>&1 || exit 1
for D in libjp2hip_debug libjp2hip_dbgmasks0; do
  JP2HIP_LIBRARY=$L/$D.so timeout -k 10 200 python tests/tools/mq_census.py > $o/census_$D.txt 2>&1 || exit 1
done
for P in libjp2hip libjp2hip_masks0; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
bash tests/tools/ab_lib.sh ${1:-r5masks}/ab $L/libjp2hip.so $L/libjp2hip_masks0.so 2 || exit 1
