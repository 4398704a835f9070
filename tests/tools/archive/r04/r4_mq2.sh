#!/bin/bash
# MQ modeller state words carrying both successors (one 8-byte read), A
# scaled by 2^16, coder ring by bit-field insert: GPU suite on the new build,
# then C2 bench alternating base / new, then one image's stage times each.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4mq2}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
for r in 1 2 3; do
for t in libjp2hip_mqbase libjp2hip_mqnew; do
  JP2HIP_LIBRARY=$L/$t.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-extras > $o/b_${t}_$r.json 2> $o/b_${t}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/b_${t}_$r.json').read().strip().splitlines()[-1]); print('$t bench $r', d['value'], d['roofline']['avg_launch_ms'], d['config'].get('single_image_latency_ms'))" | tee -a $o/summary.txt
done
done
