#!/bin/bash
# Round-end evidence on one box: GPU parity suite, MQ census, default bench
# line, rocprofv3 kernel-trace stats of the same command, and two PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of the dominant kernel.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/final
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
PYTHONPATH=jp2-bucketeer_amd timeout -k 10 120 python tests/tools/mq_census.py > $o/mq_census.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless > $o/bench_kt.json 2> $o/bench_kt.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o/pmc_fetch -o run --output-format csv -- python bench.py --steps 24 --warmup 1 --inflight 1 --no-cpu-baseline --no-lossless > $o/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o/pmc_write -o run --output-format csv -- python bench.py --steps 24 --warmup 1 --inflight 1 --no-cpu-baseline --no-lossless > $o/pmc_write.log 2>&1 || exit 1
python tests/tools/pmc_summary.py --fetch $o/pmc_fetch --write $o/pmc_write --out $o/pmc_traffic.json || exit 1
timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 > $o/bench_c5.json 2> $o/bench_c5.err || exit 1
