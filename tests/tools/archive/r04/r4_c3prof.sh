#!/bin/bash
# Lossless C3 in flight: one image's stats, a longer in-flight run, and the
# same under rocprofv3's kernel + memory-copy trace (where the time goes).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-c3prof}
mkdir -p $o
export GPU_MAX_HW_QUEUES=12
C3_EACH=6 timeout -k 10 300 python tests/tools/c3_inflight.py 4 6 8 > $o/c3.txt 2> $o/c3.err || exit 1
C3_EACH=4 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/kt -o run --output-format csv -- python tests/tools/c3_inflight.py 6 > $o/c3_prof.txt 2> $o/c3_prof.err || exit 1
python tests/tools/kstats.py $o/kt/run_kernel_stats.csv > $o/kstats.txt 2>&1 || true
python tests/tools/stream_gaps.py $o/kt/run_kernel_trace.csv > $o/stream_gaps.txt 2>&1 || true
ls $o/kt >> $o/c3.txt
