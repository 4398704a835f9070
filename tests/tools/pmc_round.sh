#!/bin/bash
# The PMC summaries bench.py cites (profiles/rNN/t1_sq_counters.json,
# pmc_traffic.json): SQ and HBM-traffic passes (one counter set per run) over
# single-image C2 encodes, GPU_MAX_HW_QUEUES as the bench sets it (16).
set -o pipefail
export TMPDIR=/tmp
o=${1:-r02}
bash tests/tools/pmc_kernels.sh pmc_$o "k_" || exit 1
python tests/tools/sq_summary.py gpurun_out/pmc_$o/p1 gpurun_out/pmc_$o/p2 --out profiles/$o/t1_sq_counters.json > gpurun_out/pmc_$o/sq.txt || exit 1
python tests/tools/pmc_summary.py --fetch gpurun_out/pmc_$o/p3 --write gpurun_out/pmc_$o/p4 --out profiles/$o/pmc_traffic.json > gpurun_out/pmc_$o/traffic.txt || exit 1
mkdir -p gpurun_out/pmc_$o/out && cp profiles/$o/t1_sq_counters.json profiles/$o/pmc_traffic.json gpurun_out/pmc_$o/out/
