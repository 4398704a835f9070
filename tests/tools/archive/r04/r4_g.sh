#!/bin/bash
# Chain-bound or capacity-bound?  The C2 bench with an extra host delay per
# encode (0 / 0.5 / 1 ms, alternating): a chain-bound pipeline slows by about
# delay / chain; a capacity-bound one does not.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4g}
mkdir -p $o
for r in 1 2; do
  for d in 0 0.5 1.0; do
    JP2HIP_BENCH_HOST_DELAY_MS=$d timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-extras > $o/b_${d}_$r.json 2> $o/b_${d}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${d}_$r.json').read().strip().splitlines()[-1]); print('delay=$d', $r, d['value'], d['ms_per_step'])" | tee -a $o/summary.txt
  done
done
