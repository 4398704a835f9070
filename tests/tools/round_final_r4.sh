#!/bin/bash
# Round-4 evidence on one MI355X: smoke + the whole GPU suite, the driver's
# bench command (every key), the C2 leg alone under rocprofv3 (queue count
# exported before the profiler starts) with the HIP-event / rocprofv3
# agreement of k_t1_mq, and single-image kernel statistics.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r04_final}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
tail -n1 $o/gpu_tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || exit 1
bash tests/tools/prof_r4.sh ${1:-r04_final}/prof || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-extras --inflight 1 --batch 1 --steps 16 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
