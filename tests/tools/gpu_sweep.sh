#!/bin/bash
# The randomized parity sweep (all cases, no -x: every divergence is listed),
# then the whole GPU suite.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-sweep}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $o/sweep.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread --deselect tests/test_gpu_sweep.py > $o/gpu_tests.log 2>&1
