#!/bin/bash
# A/B of an environment knob on the C2 bench line, alternating runs:
#   bash tests/tools/ab_env.sh OUT VAR VALUE_A VALUE_B [ROUNDS]
set -o pipefail
o=gpurun_out/$1; var=$2; va=$3; vb=$4; n=${5:-2}
mkdir -p $o
B="python bench.py --no-cpu-baseline --no-lossless --steps 10"
for i in $(seq 1 $n); do
  env $var=$va timeout -k 10 200 $B > $o/a$i.json 2> $o/a$i.err || exit 1
  env $var=$vb timeout -k 10 200 $B > $o/b$i.json 2> $o/b$i.err || exit 1
done
