#!/bin/bash
# rocprofv3 PMC passes (one counter set per run) over single-image C2 encodes,
# every jp2hip kernel: SQ instruction / wait counters, HBM bytes, and the
# instruction-cache counters.  Summaries land in profiles/<round>/.
#   tests/tools/pmc_all.sh <round> [kernel regex]
set -o pipefail
export TMPDIR=/tmp
r=${1:-r04}
re=${2:-"k_"}
o=gpurun_out/pmc_$r
mkdir -p $o profiles/$r
B="python bench.py --inflight 1 --steps 3 --warmup 1 --no-extras"
P() { timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-include-regex "$re" -d $o/$1 -o run --output-format csv -- $B > $o/$1.log 2>&1; }
P p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" || exit 1
P p2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" || exit 1
P p3 FETCH_SIZE || exit 1
P p4 WRITE_SIZE || exit 1
P p5 "SQC_ICACHE_HITS SQC_ICACHE_MISSES GRBM_GUI_ACTIVE" || exit 1
python tests/tools/sq_summary.py $o/p1 $o/p2 $o/p5 --out profiles/$r/t1_sq_counters.json > $o/sq.txt || exit 1
python tests/tools/pmc_summary.py --fetch $o/p3 --write $o/p4 --out profiles/$r/pmc_traffic.json > $o/traffic.txt || exit 1
mkdir -p $o/out && cp profiles/$r/t1_sq_counters.json profiles/$r/pmc_traffic.json $o/out/
