#!/bin/bash
# Big single-context images (F x F C2 images, one stream) and the SQ wave
# counters of the block-sequential k_t1_cm3 against the item kernel.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4i}
mkdir -p $o
timeout -k 10 300 python -u tests/tools/big_image.py 2 > $o/big2.txt 2>&1 || exit 1
timeout -k 10 300 python -u tests/tools/big_image.py 4 > $o/big4.txt 2>&1 || exit 1
L=jp2-bucketeer_amd/jp2hip
B="python bench.py --inflight 1 --steps 3 --warmup 1 --no-extras"
for t in libjp2hip_items libjp2hip; do
  JP2HIP_LIBRARY=$L/$t.so timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex k_t1_cm3 -d $o/p1_$t -o run --output-format csv -- $B > $o/p1_$t.log 2>&1 || exit 1
  python tests/tools/sq_summary.py $o/p1_$t --out $o/sq_$t.json > /dev/null || exit 1
done
