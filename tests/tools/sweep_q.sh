#!/bin/bash
# default bench (12 in flight, 12 HW queues) vs 4 HW queues, interleaved
out=gpurun_out/sweep_q.txt
: > $out
for rep in 1 2 3; do
  for q in 12 4 16; do
    r=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu-baseline --no-lossless --inflight 12 --steps 192) || exit 1
    v=$(echo "$r" | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['stages_ms']['total_ms'])")
    echo "rep $rep queues $q value $v" | tee -a $out
  done
done
