#!/bin/bash
# Round 6 evidence set on one GPU box: the C2 leg under rocprofv3 (kernel
# stats under load, HIP-event / rocprofv3 agreement of k_t1_mq, stream
# gaps), one image at a time (alone durations), PMC traffic + SQ counters
# (profiles/r06/*.json, which bench.py cites), and a C3 in-flight run under
# rocprofv3 (where the lossless production image's GPU time goes).
#   tests/tools/r6_evidence.sh <out-name>
set -o pipefail
export TMPDIR=/tmp
o=${1:-r6ev}
bash tests/tools/prof_r4.sh $o/prof || exit 1
export GPU_MAX_HW_QUEUES=8 JP2HIP_KEEP_HW_QUEUES=1
mkdir -p gpurun_out/$o
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$o/kt1 -o run --output-format csv -- python bench.py --no-extras --inflight 1 --batch 1 --steps 12 --warmup 2 > gpurun_out/$o/bench_kt1.json 2> gpurun_out/$o/bench_kt1.err || exit 1
python tests/tools/kstats.py gpurun_out/$o/kt1/run_kernel_stats.csv > gpurun_out/$o/kstats_single.txt 2>&1 || true
unset GPU_MAX_HW_QUEUES JP2HIP_KEEP_HW_QUEUES
bash tests/tools/pmc_round.sh r06 || exit 1
export GPU_MAX_HW_QUEUES=12 JP2HIP_KEEP_HW_QUEUES=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$o/c3 -o run --output-format csv -- python tests/tools/c3_inflight.py 8 > gpurun_out/$o/c3_inflight.jsonl 2> gpurun_out/$o/c3_inflight.err || exit 1
python tests/tools/kstats.py gpurun_out/$o/c3/run_kernel_stats.csv > gpurun_out/$o/c3_kstats.txt 2>&1 || true
