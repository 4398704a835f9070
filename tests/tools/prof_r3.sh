#!/bin/bash
# Round-3 profile set: single-image kernel trace, SQ counter passes over
# single-image encodes, and an in-flight sweep of the C2 bench.
#   tests/tools/prof_r3.sh <out-name> [sweep values...]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-p3}
shift
mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --batch 1 --steps 12 --warmup 2 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
bash tests/tools/pmc_kernels.sh $(basename $o)/pmc "k_dwt|k_quant|k_t1_cm3|k_t1_mq|k_t2_code|k_select|k_hull" || exit 1
for n in "$@"; do
  timeout -k 10 200 python bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-lossless --inflight $n > $o/if$n.json 2> $o/if$n.err || exit 1
done
