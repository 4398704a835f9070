#!/bin/bash
out=gpurun_out/sweep_q3.txt
: > $out
for rep in 1 2 3; do
  for cfg in "12 16" "12 4" "12 8" "8 12"; do
    set -- $cfg
    r=$(GPU_MAX_HW_QUEUES=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --no-lossless --inflight $1 --steps 144) || exit 1
    v=$(echo "$r" | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['stages_ms']['total_ms'], d['stages_ms']['t2_ms'])")
    echo "rep $rep inflight $1 queues $2 value $v" | tee -a $out
  done
done
nproc; lscpu | grep -i "model name"
