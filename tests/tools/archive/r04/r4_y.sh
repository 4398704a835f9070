#!/bin/bash
# bench.py with the worker's Python work trimmed (product) vs the previous
# worker (bench_prev.py), same library: C2 bench, alternating.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4y}
mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_gpu_api.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
tail -n1 $o/t.log
for r in 1 2 3; do
for b in bench_prev bench; do
  timeout -k 10 240 python $b.py --steps 16 --warmup 2 --no-extras > $o/${b}_$r.json 2> $o/${b}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/${b}_$r.json').read().strip().splitlines()[-1]); print('$b run $r', d['value'])" | tee -a $o/summary.txt
done
done
