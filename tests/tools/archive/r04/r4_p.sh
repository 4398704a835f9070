#!/bin/bash
# DWT band kernel: 128-thread workgroups for levels <= 128 wide (product)
# vs 256 always (base), and 16 kept rows per workgroup (rb16): parity
# subset, then kernel times + bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4p}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
tail -1 $o/t.log
JP2HIP_LIBRARY=$L/libjp2hip_rb16.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t_rb16.log 2>&1 || exit 1
tail -1 $o/t_rb16.log
AB_ROUNDS=2 bash tests/tools/ab_kt.sh ${1:-r4p}/ab $L/libjp2hip_base.so $L/libjp2hip.so $L/libjp2hip_rb16.so || exit 1
