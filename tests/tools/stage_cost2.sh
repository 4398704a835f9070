#!/bin/bash
# Marginal cost of each stage under the bench's load: the C2 bench with one
# stage's kernels launched twice (libjp2hip_rep<n>.so, built with
# -DJP2HIP_REPEAT_STAGE=<n>), against the product library, alternating.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-stagecost}
mkdir -p $o
for r in 1 2; do
  for L in libjp2hip libjp2hip_rep1 libjp2hip_rep2 libjp2hip_rep3 libjp2hip_rep4 libjp2hip_rep5; do
    JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/$L.so timeout -k 10 200 python bench.py --steps 16 --warmup 2 --no-extras > $o/${L}_$r.json 2> $o/${L}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/${L}_$r.json').read().strip().splitlines()[-1]); print('$L', $r, d['value'], round(16*24/d['value']*1e3/16,4), d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
