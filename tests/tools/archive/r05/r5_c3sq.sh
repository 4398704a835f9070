#!/bin/bash
# SQ instruction counters of one C2 and one C3 image per kernel
# (tests/tools/mq_alone.py encodes each 6 times), one counter set per pass.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3sq}
mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "k_" -d $o/p1 -o run --output-format csv -- python tests/tools/mq_alone.py > $o/p1.log 2>&1 || exit 1
