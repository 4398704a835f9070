#!/bin/bash
# A/B of two builds: parity subset on the in-tree build, one image alone
# (HIP events) and the C2 bench, alternating.  r4_ab3.sh <out> <libA> <libB>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-ab3}; A=$2; B=$3
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -1 $o/gpu_tests.log | tee -a $o/summary.txt
for r in 1 2; do
for t in $A $B; do
  JP2HIP_LIBRARY=$L/$t.so timeout -k 10 200 python tests/tools/mq_alone.py >> $o/summary.txt 2> $o/$t.err || exit 1
done
done
for r in 1 2 3; do
for t in $A $B; do
  JP2HIP_LIBRARY=$L/$t.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-extras > $o/b_${t}_$r.json 2> $o/b_${t}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/b_${t}_$r.json').read().strip().splitlines()[-1]); print('$t bench $r', d['value'], d['roofline']['avg_launch_ms'], d['config'].get('single_image_latency_ms'))" | tee -a $o/summary.txt
done
done
