#!/bin/bash
# k_hull's slope-bin histogram in HBM directly, no LDS (product) vs the
# 32 KB LDS workgroup histogram (hlds): parity on the product, C2 bench, the
# C2 leg under rocprofv3 for both (rate-loop kernels under load), one image
# at a time for both.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5hlds}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_split_native.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/parity.txt 2>&1 || exit 1
for r in 1 2; do
  for P in libjp2hip libjp2hip_hlds; do
    JP2HIP_LIBRARY=$L/$P.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${P}_$r.json 2> $o/b_${P}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$o/b_${P}_$r.json').read().strip().splitlines()[-1]); print('$P', $r, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
  done
done
for P in libjp2hip libjp2hip_hlds; do
  JP2HIP_LIBRARY=$L/$P.so bash tests/tools/prof_r4.sh $(basename $o)/prof_$P || exit 1
done
export GPU_MAX_HW_QUEUES=8 JP2HIP_KEEP_HW_QUEUES=1
for P in libjp2hip libjp2hip_hlds; do
  JP2HIP_LIBRARY=$L/$P.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt1_$P -o run --output-format csv -- python bench.py --no-extras --inflight 1 --batch 1 --steps 24 --warmup 4 > $o/bench_kt1_$P.json 2> $o/bench_kt1_$P.err || exit 1
  python tests/tools/kstats.py $o/kt1_$P/run_kernel_stats.csv > $o/kstats_single_$P.txt 2>&1 || true
done
