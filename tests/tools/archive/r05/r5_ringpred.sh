#!/bin/bash
# k_t1_cm3's ring writer: atomics only on the dwords a lane's bytes reach
# (product) vs every lane OR-ing all NW dwords (rp0): parity, stage times
# alone (C2, C3), C2 bench, C3 in flight, SQ LDS counters of k_t1_cm3.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5ringp}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
for P in libjp2hip libjp2hip_rp0; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
for r in 1 2; do
  for P in libjp2hip libjp2hip_rp0; do
    JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${P}_$r.json 2> $o/b_${P}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${P}_$r.json').read().strip().splitlines()[-1]); print('$P', $r, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
for P in libjp2hip libjp2hip_rp0; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python tests/tools/c3_inflight.py 8 > $o/c3_$P.txt 2>&1 || exit 1
done
for P in libjp2hip libjp2hip_rp0; do
  JP2HIP_LIBRARY=$L/$P.so timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU --kernel-include-regex "k_t1_cm3" -d $o/pmc_$P -o run --output-format csv -- python tests/tools/mq_alone.py > $o/pmc_$P.log 2>&1 || exit 1
done
