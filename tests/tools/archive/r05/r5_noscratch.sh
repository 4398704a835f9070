#!/bin/bash
# The pass prefetch's plane-count load as a global load with a value select
# (was a flat load from a selected address: `cnt` in scratch) and the DWT's
# row quantisers selected as register values (were scratch loads): product
# vs the previous build (old): parity, census, stage times, C2 bench, C3 in
# flight.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5noscr}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/parity.txt 2>&1 || exit 1
for D in libjp2hip_debug libjp2hip_dbgold; do
  JP2HIP_LIBRARY=$L/$D.so timeout -k 10 200 python tests/tools/mq_census.py > $o/census_$D.txt 2>&1 || exit 1
done
for P in libjp2hip libjp2hip_old; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
for r in 1 2; do
  for P in libjp2hip libjp2hip_old; do
    JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${P}_$r.json 2> $o/b_${P}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${P}_$r.json').read().strip().splitlines()[-1]); print('$P', $r, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
for P in libjp2hip libjp2hip_old; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python tests/tools/c3_inflight.py 8 > $o/c3_$P.txt 2>&1 || exit 1
done
