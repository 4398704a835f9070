#!/bin/bash
# in-flight x HW-queue sweep (blocking-sync build), interleaved
out=gpurun_out/sweep_q2.txt
: > $out
for rep in 1 2; do
  for cfg in "12 16" "16 16" "16 24" "24 24" "32 32"; do
    set -- $cfg
    r=$(GPU_MAX_HW_QUEUES=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --no-lossless --inflight $1 --steps $(( $1 * 16 ))) || exit 1
    v=$(echo "$r" | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['stages_ms']['total_ms'])")
    echo "rep $rep inflight $1 queues $2 value $v" | tee -a $out
  done
done
