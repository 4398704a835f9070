#!/bin/bash
# DMA engines vs blit kernels for the code-stream D2H under the bench's load:
# the C2 bench with HSA_ENABLE_SDMA=0 / 1 alternating, then a kernel trace of
# the SDMA run (does __amd_rocclr_copyBuffer still appear?)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-sdma}
mkdir -p $o
env | grep -iE "sdma|^hsa_|^hip_|^roc" > $o/env.txt
B="python bench.py --no-cpu-baseline --no-lossless --steps 16 --warmup 2"
for i in 1 2; do
  HSA_ENABLE_SDMA=0 timeout -k 10 200 $B > $o/a$i.json 2> $o/a$i.err || exit 1
  HSA_ENABLE_SDMA=1 timeout -k 10 200 $B > $o/b$i.json 2> $o/b$i.err || exit 1
  python -c "
import json
for t in 'ab':
    d=json.loads(open('$o/'+t+'$i.json').read().strip().splitlines()[-1]); print(t, $i, d['value'], d['config']['single_image_latency_ms'])" | tee -a $o/summary.txt
done
HSA_ENABLE_SDMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --steps 8 --warmup 2 > $o/kt.json 2> $o/kt.err || exit 1
