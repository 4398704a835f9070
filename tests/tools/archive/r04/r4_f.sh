#!/bin/bash
# Does per-stage event recording (profile mode) cost throughput under load?
# Alternating C2-only benches with JP2HIP_BENCH_PROFILE=1 / 0.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4f}
mkdir -p $o
for r in 1 2 3; do
  for pr in 1 0; do
    JP2HIP_BENCH_PROFILE=$pr timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-extras > $o/b_${pr}_$r.json 2> $o/b_${pr}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${pr}_$r.json').read().strip().splitlines()[-1]); print('profile=$pr', $r, d['value'])" | tee -a $o/summary.txt
  done
done
