#!/bin/bash
# A/B of two library builds on one box: the C2 bench line, alternating.
set -o pipefail
o=gpurun_out/${1:-ab}
mkdir -p $o
B="python bench.py --no-cpu-baseline --no-lossless --steps 48"
for r in 1 2; do
  for v in old new; do
    JP2HIP_LIBRARY=$PWD/exp/libjp2hip_$v.so timeout -k 10 200 $B > $o/$v$r.json 2> $o/$v$r.err || exit 1
  done
done
