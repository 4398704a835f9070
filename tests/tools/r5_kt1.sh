#!/bin/bash
# Single-image kernel statistics of the C2 leg (one context, one image at a
# time), as r5_round.sh's last step.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5kt1}
mkdir -p $o
export GPU_MAX_HW_QUEUES=8 JP2HIP_KEEP_HW_QUEUES=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-extras --inflight 1 --batch 1 --steps 24 --warmup 4 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
python tests/tools/kstats.py $o/kt1/run_kernel_stats.csv > $o/kstats_single.txt 2>&1 || true
