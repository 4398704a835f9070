#!/bin/bash
# SQ LDS counters of k_dwt_l1s for two builds (single-image C2 encodes)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r06_sq
mkdir -p $o
for L in jp2-bucketeer_amd/jp2hip/libjp2hip_noskew.so jp2-bucketeer_amd/jp2hip/libjp2hip.so; do
  t=$(basename $L .so)
  JP2HIP_LIBRARY=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "k_dwt_l1s" -d $o/$t -o run --output-format csv -- python bench.py --inflight 1 --steps 3 --warmup 1 --no-extras > $o/$t.log 2>&1 || exit 1
done
