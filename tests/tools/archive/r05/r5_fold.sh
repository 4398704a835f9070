#!/bin/bash
# GPU suite, then single-image kernel times and the C2 bench of the product
# against its A/B variants (tests/tools/ab_kt.sh).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5fold}; shift
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.txt 2>&1 || exit 1
bash tests/tools/ab_kt.sh $(basename $o)/kt "$@" || exit 1
