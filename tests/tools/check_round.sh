#!/bin/bash
# One GPU check of the current tree: smoke, the GPU parity suite, a short
# bench and a rocprofv3 kernel-stats run of the same bench.
#   tests/tools/check_round.sh <out-name> [bench args...]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-chk}
shift
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-lossless "$@" > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-lossless "$@" > $o/bench_rocprof.json 2> $o/bench_rocprof.err || exit 1
