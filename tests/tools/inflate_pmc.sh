#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/infpmc
mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_inflate" -d $o/p1 -o run --output-format csv -- python tests/tools/inflate_pmc.py > $o/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU --kernel-include-regex "k_inflate" -d $o/p2 -o run --output-format csv -- python tests/tools/inflate_pmc.py > $o/p2.log 2>&1 || exit 1
python tests/tools/sq_summary.py $o/p1 $o/p2 --out $o/inflate_sq.json
