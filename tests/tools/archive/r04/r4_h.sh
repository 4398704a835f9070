#!/bin/bash
# k_t1_cm3 one wave per block (planes in order) vs per (block, plane) item: parity (sweep + parity
# suite subset), then kernel times + bench against the previous build (base).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4h}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
tail -1 $o/t.log
AB_ROUNDS=3 bash tests/tools/ab_kt.sh ${1:-r4h}/ab $L/libjp2hip_items.so $L/libjp2hip.so || exit 1
