#!/bin/bash
# A/B of two library builds on the C2 bench (alternating, n rounds):
#   tests/tools/ab_lib.sh <out-name> <libA.so> <libB.so> [rounds] [bench args]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-ab}; A=$2; B=$3; n=${4:-2}; shift 4
mkdir -p $o
for i in $(seq $n); do
  for L in $A $B; do
    t=$(basename $L .so)
    JP2HIP_LIBRARY=$L timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless "$@" > $o/${t}_$i.json 2> $o/${t}_$i.err || exit 1
    python -c "import json; d=json.loads(open('$o/${t}_$i.json').read().strip().splitlines()[-1]); print('$t', $i, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
