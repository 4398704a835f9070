#!/bin/bash
# GPU parity suite + smoke; if green, the C2 bench line and a rocprofv3
# kernel trace of single-image C2 encodes (kernel durations alone).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-gtp}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 48 > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --steps 16 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
