#!/bin/bash
# Ring writer with guard words / constant-offset atomics: parity subset,
# then the resource probe (r4_j.sh) against it.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4k}
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
tail -1 $o/t.log
bash tests/tools/r4_j.sh ${1:-r4k}/probe || exit 1
