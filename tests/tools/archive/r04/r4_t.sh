#!/bin/bash
# Images in flight per GPU (hardware queues = in flight + 4): 12 / 16 / 20 / 24.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4t}
mkdir -p $o
for r in 1 2; do
for n in 12 16 20 24; do
  timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-extras --inflight $n > $o/b_${n}_$r.json 2> $o/b_${n}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/b_${n}_$r.json').read().strip().splitlines()[-1]); print('inflight $n run $r', d['value'], d['config']['hw_queues'])" | tee -a $o/summary.txt
done
done
