#!/bin/bash
# Round-end evidence (third pass, k_t1_mq timed by its own wall-clock span):
# smoke, GPU parity suite, default bench line, and the rocprofv3 kernel-trace
# stats of the same bench command (its JSON line beside), plus C4 / C5 lines.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/final3
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless > $o/bench_kt.json 2> $o/bench_kt.err || exit 1
timeout -k 10 300 python bench.py --workload c4 --steps 96 > $o/bench_c4.json 2> $o/bench_c4.err || exit 1
timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 > $o/bench_c5.json 2> $o/bench_c5.err || exit 1
