#!/bin/bash
# Interleaved in-flight / HW-queue sweep on one box (noise control): three
# rounds over the same configurations, one line per run.
out=gpurun_out/sweep.txt
: > $out
for rep in 1 2 3; do
  for cfg in "6 4" "8 8" "12 12" "16 16"; do
    set -- $cfg
    r=$(GPU_MAX_HW_QUEUES=$2 timeout -k 10 120 python bench.py --inflight $1 --steps $(( $1 * 24 )) --warmup 1 --no-cpu-baseline --no-lossless) || exit 1
    v=$(echo "$r" | python -c "import json,sys; print(json.load(sys.stdin)['value'])")
    echo "rep $rep inflight $1 queues $2 value $v" | tee -a $out
  done
done
