#!/bin/bash
# PCRD-opt hulls in k_t1_mq's tail (product; k_hull launch gone) vs the
# previous build (prevh): GPU suite on the product, stage times alone, C2
# bench, C3 in flight, then the product's C2 leg under rocprofv3 (rate-loop
# kernels under load) and one image at a time.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5hull}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
for P in libjp2hip libjp2hip_prevh; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$P.txt 2>&1 || exit 1
done
for r in 1 2; do
  for P in libjp2hip libjp2hip_prevh; do
    JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${P}_$r.json 2> $o/b_${P}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${P}_$r.json').read().strip().splitlines()[-1]); print('$P', $r, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
for P in libjp2hip libjp2hip_prevh; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python tests/tools/c3_inflight.py 8 > $o/c3_$P.txt 2>&1 || exit 1
done
JP2HIP_LIBRARY=$L/libjp2hip_debug.so timeout -k 10 200 python tests/tools/mq_census.py > $o/mq_census.txt 2>&1 || exit 1
bash tests/tools/prof_r4.sh $(basename $o)/prof || exit 1
export GPU_MAX_HW_QUEUES=8 JP2HIP_KEEP_HW_QUEUES=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-extras --inflight 1 --batch 1 --steps 24 --warmup 4 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
python tests/tools/kstats.py $o/kt1/run_kernel_stats.csv > $o/kstats_single.txt 2>&1 || true
