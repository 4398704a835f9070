#!/bin/bash
# k_t1_cm3 blocks pipelined one ahead (descriptor + first masks): parity
# (parity suite, sweep, native split), then kernel times + bench vs HEAD (base).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4w}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_split_native.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
tail -1 $o/t.log
AB_ROUNDS=3 bash tests/tools/ab_kt.sh ${1:-r4w}/ab $L/libjp2hip_base.so $L/libjp2hip.so || exit 1
