#!/bin/bash
# A/B of two library builds: single-image k_t1_mq time (rocprofv3 kernel
# stats) and the C2 bench, alternating.
#   tests/tools/ab_mq.sh <out-name> <libA.so> <libB.so>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-abmq}; A=$2; B=$3
mkdir -p $o
for L in $A $B; do
  t=$(basename $L .so)
  JP2HIP_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt_$t -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --batch 1 --steps 8 --warmup 2 > $o/kt_$t.json 2> $o/kt_$t.err || exit 1
  grep -E "k_t1_mq|k_t1_cm3" $o/kt_$t/run_kernel_stats.csv | cut -d, -f1,4 | sed "s/^/$t /" | tee -a $o/summary.txt
done
bash tests/tools/ab_lib.sh $1 $A $B 2 || exit 1
