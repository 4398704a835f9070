#!/bin/bash
# C3 images in flight: 4 .. 12 contexts, twice.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3s}
mkdir -p $o
for r in 1 2; do
  C3_EACH=3 timeout -k 10 400 python tests/tools/c3_inflight.py 4 6 8 10 12 > $o/sweep_$r.json 2> $o/sweep_$r.err || exit 1
done
