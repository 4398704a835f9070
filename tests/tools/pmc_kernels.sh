#!/bin/bash
# rocprofv3 PMC passes (one counter set per run, as the pool requires) over
# single-image C2 encodes: SQ instruction / wait / LDS counters and HBM bytes
# for the front-end kernels (DWT, quantiser, tier-1).  GPU_MAX_HW_QUEUES is
# set here, in the environment rocprofv3 hands to bench.py, to the value
# bench.py itself uses for 12 contexts (16).
set -o pipefail
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16 JP2HIP_KEEP_HW_QUEUES=1
o=gpurun_out/${1:-pmc}
re=${2:-"k_dwt|k_quant|k_t1_cm|k_t1_mq"}
mkdir -p $o
B="python bench.py --inflight 1 --steps 3 --warmup 1 --no-extras"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "$re" -d $o/p1 -o run --output-format csv -- $B > $o/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --kernel-include-regex "$re" -d $o/p2 -o run --output-format csv -- $B > $o/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$re" -d $o/p3 -o run --output-format csv -- $B > $o/p3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$re" -d $o/p4 -o run --output-format csv -- $B > $o/p4.log 2>&1 || exit 1
