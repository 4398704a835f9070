#!/bin/bash
# Round-end evidence on one MI355X: smoke + the GPU suite, the driver's bench
# command (CPU baseline included), the same command under rocprofv3 kernel
# trace + stats, and a kernel trace of single-image encodes.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-final}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $o/bench_rocprof.json 2> $o/bench_rocprof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --batch 1 --steps 16 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
