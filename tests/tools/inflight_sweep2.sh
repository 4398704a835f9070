#!/bin/bash
# C2 throughput vs (images in flight, hardware queues, stage profiling):
#   tests/tools/inflight_sweep2.sh <out-name> "inflight:hwq:profile ..."
set -o pipefail
export TMPDIR=/tmp JP2HIP_KEEP_HW_QUEUES=1
o=gpurun_out/${1:-sweep2}
mkdir -p $o
for c in $2; do
  IFS=: read nf q pf <<< "$c"
  GPU_MAX_HW_QUEUES=$q JP2HIP_BENCH_PROFILE=$pf timeout -k 10 240 python bench.py --steps 16 --warmup 2 --inflight $nf \
      --no-cpu-baseline --no-lossless > $o/if${nf}_q${q}_p${pf}.json 2> $o/if${nf}_q${q}_p${pf}.err || exit 1
  python -c "import json,sys; d=json.loads(open('$o/if${nf}_q${q}_p${pf}.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'])" | tee -a $o/summary.txt
done
