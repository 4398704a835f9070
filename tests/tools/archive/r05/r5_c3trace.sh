#!/bin/bash
# Lossless C3 with 6 contexts in flight under a kernel + memory-copy trace:
# per-kernel busy time, concurrency and per-stream gaps (tests/tools/
# trace_busy.py, stream_gaps.py read the CSVs).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3t}
mkdir -p $o
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/kt -o run --output-format csv -- python tests/tools/c3_inflight.py 6 > $o/c3.json 2> $o/c3.err || exit 1
