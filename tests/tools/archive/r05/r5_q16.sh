#!/bin/bash
# Quantisation indices written by the DWT (16-bit plane) and the S masks no
# longer stored: GPU suite, single-image stage times and C2 bench against the
# previous build, whole-path HBM traffic (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5q16}
B=${2:-jp2-bucketeer_amd/jp2hip/libjp2hip_masks0.so}
L=jp2-bucketeer_amd/jp2hip/libjp2hip.so
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.txt 2>&1 || exit 1
for P in $L $B; do
  JP2HIP_LIBRARY=$P timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$(basename $P .so).txt 2>&1 || exit 1
done
bash tests/tools/ab_lib.sh ${1:-r5q16}/ab $L $B 2 || exit 1
export GPU_MAX_HW_QUEUES=16 JP2HIP_KEEP_HW_QUEUES=1
C="python bench.py --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline --no-lossless"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_" -d $o/p3 -o run --output-format csv -- $C > $o/p3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_" -d $o/p4 -o run --output-format csv -- $C > $o/p4.log 2>&1 || exit 1
python tests/tools/pmc_summary.py --fetch $o/p3 --write $o/p4 --out $o/pmc_traffic.json > $o/traffic.txt || exit 1
