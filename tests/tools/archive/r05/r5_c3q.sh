#!/bin/bash
# C3 in flight (8 contexts) standalone with 12 and with 20 hardware queues,
# then the bench's own lossless leg after its C2 leg (20 queues).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3q}
mkdir -p $o
for q in 12 20 12 20; do
  GPU_MAX_HW_QUEUES=$q JP2HIP_KEEP_HW_QUEUES=1 C3_EACH=4 timeout -k 10 300 python tests/tools/c3_inflight.py 8 > $o/c3_q$q.json 2> $o/c3_q$q.err || exit 1
  echo "q$q $(grep inflight $o/c3_q$q.json)" | tee -a $o/summary.txt
done
timeout -k 10 600 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > $o/bench.json 2> $o/bench.err || exit 1
python -c "import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]); print('bench c3', d['lossless_c3']['mp_per_s_inflight_c_api'])" | tee -a $o/summary.txt
