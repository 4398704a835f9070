#!/bin/bash
# A/B: DWT level-1 stream band 32 rows (sb32), MQ 32-byte rings (ring32) --
# parity of each variant on a few GPU cases first, then kernel times + bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4d}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
for v in sb32 ring32; do
  JP2HIP_LIBRARY=$L/libjp2hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "codestream_identical or golden_lossy or smoke_image or sweep_identical" > $o/t_$v.log 2>&1 || exit 1
  tail -1 $o/t_$v.log
done
AB_ROUNDS=3 bash tests/tools/ab_kt.sh ${1:-r4d}/ab $L/libjp2hip.so $L/libjp2hip_sb32.so $L/libjp2hip_ring32.so || exit 1
