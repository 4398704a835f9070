#!/bin/bash
# k_t1_cm3 register budget: the product (105 VGPRs, 4 waves per SIMD) vs
# waves_per_eu 5 (95 VGPRs, 5 spill slots) and 6 (80 VGPRs, 13): stage
# times alone, C2 bench, C3 in flight; parity on the 5-wave build.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5cmwpe}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
for P in libjp2hip libjp2hip_cmw5 libjp2hip_cmw6; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
for r in 1 2; do
  for P in libjp2hip libjp2hip_cmw5 libjp2hip_cmw6; do
    JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${P}_$r.json 2> $o/b_${P}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${P}_$r.json').read().strip().splitlines()[-1]); print('$P', $r, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
for P in libjp2hip libjp2hip_cmw5 libjp2hip_cmw6; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python tests/tools/c3_inflight.py 8 > $o/c3_$P.txt 2>&1 || exit 1
done
JP2HIP_LIBRARY=$L/libjp2hip_cmw5.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/parity_cmw5.txt 2>&1 || exit 1
