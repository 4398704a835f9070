#!/bin/bash
# SQ occupancy / VALU counters of the tier-1 kernels (one image in flight so
# the counters belong to one kernel at a time), then the default bench line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/sq
mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "k_t1_(mq|cm)" -d $o/pmc -o run --output-format csv -- python bench.py --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline --no-lossless > $o/pmc.log 2>&1 || exit 1
python tests/tools/sq_summary.py $o/pmc --out profiles/r01/t1_sq_counters.json > $o/sq_summary.txt || exit 1
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err || exit 1
