#!/bin/bash
# Marginal cost of each front-end stage under the bench's load: the C2 bench
# line with that stage's kernel launched twice (JP2HIP_REPEAT_STAGE).
set -o pipefail
o=gpurun_out/${1:-stage}
mkdir -p $o
B="python bench.py --no-cpu-baseline --no-lossless --steps 8"
timeout -k 10 200 $B > $o/base.json 2> $o/base.err || exit 1
for st in mq cm quant dwt pcrd t2; do
  JP2HIP_REPEAT_STAGE=$st timeout -k 10 200 $B > $o/$st.json 2> $o/$st.err || exit 1
done
