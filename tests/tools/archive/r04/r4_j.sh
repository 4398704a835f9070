#!/bin/bash
# Resource probe: the C2 bench with k_t1_cm3 burning VALU (libjp2hip_burnv:
# ~1000 dependent VALU per plane) or idling (libjp2hip_burns: s_sleep per
# plane) against the product build -- which resource the load is bound by.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4j}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
for r in 1 2; do
for t in libjp2hip libjp2hip_burnv libjp2hip_burns; do
  JP2HIP_LIBRARY=$L/$t.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-extras > $o/b_${t}_$r.json 2> $o/b_${t}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/b_${t}_$r.json').read().strip().splitlines()[-1]); print('$t bench $r', d['value'], d['config']['single_image_latency_ms'], d['stages_ms']['t1_cm_ms'])" | tee -a $o/summary.txt
done
done
