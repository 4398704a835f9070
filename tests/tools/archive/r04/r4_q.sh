#!/bin/bash
# k_dwt_l1s horizontal batches of 8 rows (libjp2hip_l1s8) vs 4 (product):
# parity subset on the variant, then kernel times + bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4q}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
JP2HIP_LIBRARY=$L/libjp2hip_l1s8.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
tail -n1 $o/t.log
AB_ROUNDS=3 bash tests/tools/ab_kt.sh ${1:-r4q}/ab $L/libjp2hip.so $L/libjp2hip_l1s8.so || exit 1
