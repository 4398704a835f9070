#!/bin/bash
# GPU parity suite + smoke, then (if green) a short C2 bench line.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-gtb}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 48 > $o/bench.json 2> $o/bench.err || exit 1
