#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r06_mix
mkdir -p $o
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES --kernel-include-regex "k_dwt_l1s" -d $o/p1 -o run --output-format csv -- python bench.py --inflight 1 --steps 3 --warmup 1 --no-extras > $o/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM --kernel-include-regex "k_dwt_l1s" -d $o/p2 -o run --output-format csv -- python bench.py --inflight 1 --steps 3 --warmup 1 --no-extras > $o/p2.log 2>&1 || exit 1
