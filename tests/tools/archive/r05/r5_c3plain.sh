#!/bin/bash
# C3 in flight without a profiler, then under a kernel trace only.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3p}
mkdir -p $o
JP2HIP_LOG_POOL=1 timeout -k 10 300 python tests/tools/c3_inflight.py 6 > $o/plain.json 2> $o/plain.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d $o/kt -o run --output-format csv -- python tests/tools/c3_inflight.py 6 > $o/kt.json 2> $o/kt.err || exit 1
