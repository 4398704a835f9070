#!/bin/bash
# Host wait: sleeping on a blocking-sync event (product) vs polling the event
# every 20 / 100 us (libjp2hip_poll20 / poll100): C2 bench, alternating.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4o}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
for r in 1 2 3; do
for t in libjp2hip libjp2hip_poll20 libjp2hip_poll100; do
  JP2HIP_LIBRARY=$L/$t.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-extras > $o/b_${t}_$r.json 2> $o/b_${t}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/b_${t}_$r.json').read().strip().splitlines()[-1]); print('$t bench $r', d['value'])" | tee -a $o/summary.txt
done
done
