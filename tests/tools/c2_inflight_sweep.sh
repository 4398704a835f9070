#!/bin/bash
set -o pipefail
o=gpurun_out/r06_c2sw
mkdir -p $o
for r in 1 2; do
for n in 12 16 20 24; do
  timeout -k 10 200 python bench.py --no-extras --inflight $n --steps 20 --warmup 5 > $o/b_${n}_$r.json 2> $o/b_${n}_$r.err || exit 1
  python3 -c "import json; d=json.loads(open('$o/b_${n}_$r.json').read().strip().splitlines()[-1]); print($n, $r, d['value'], d['config']['hw_queues'])" | tee -a $o/summary.txt
done
done
