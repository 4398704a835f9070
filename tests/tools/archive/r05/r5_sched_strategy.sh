#!/bin/bash
# LLVM AMDGPU machine-scheduler strategies for the whole library: the product
# (default) vs max-ilp, max-memory-clause, iterative-ilp, iterative-minreg:
# stage times alone (C2, C3), C2 bench x2; parity on the best is run later.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5strat}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
V="libjp2hip libjp2hip_smilp libjp2hip_smmc libjp2hip_siilp libjp2hip_simr"
for P in $V; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
for r in 1 2; do
  for P in $V; do
    JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${P}_$r.json 2> $o/b_${P}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${P}_$r.json').read().strip().splitlines()[-1]); print('$P', $r, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
