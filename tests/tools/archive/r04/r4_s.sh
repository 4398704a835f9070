#!/bin/bash
# HEAD (base) vs the cm3 SPP-sum skip (product) vs + l1s select-free interior
# lifting at 98 VGPRs (interior): bench only, alternating.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4s}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
for r in 1 2 3; do
for t in libjp2hip_base libjp2hip libjp2hip_interior; do
  JP2HIP_LIBRARY=$L/$t.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-extras > $o/b_${t}_$r.json 2> $o/b_${t}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/b_${t}_$r.json').read().strip().splitlines()[-1]); print('$t bench $r', d['value'])" | tee -a $o/summary.txt
done
done
