#!/bin/bash
# k_t1_cm3's ring writer: the third and fourth atomics only when a lane's
# bytes reach those dwords (rpp) vs every lane OR-ing all NW dwords (the
# product): parity + sweep on rpp, stage times alone (C2, C3), C2 bench, C3
# in flight.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5ringp2}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
JP2HIP_LIBRARY=$L/libjp2hip_rpp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/parity_rpp.txt 2>&1 || exit 1
for P in libjp2hip libjp2hip_rpp; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
for r in 1 2; do
  for P in libjp2hip libjp2hip_rpp; do
    JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${P}_$r.json 2> $o/b_${P}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${P}_$r.json').read().strip().splitlines()[-1]); print('$P', $r, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
for P in libjp2hip libjp2hip_rpp; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python tests/tools/c3_inflight.py 8 > $o/c3_$P.txt 2>&1 || exit 1
done
