#!/bin/bash
# Lossless C3 in flight (6 contexts) under the HIP runtime's copy-engine
# settings: which engine carries the code-stream D2H, and the throughput.
set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
o=gpurun_out/${1:-blit}
mkdir -p $o
for v in unset 2 1 3; do
  if [ $v = unset ]; then unset GPU_BLIT_ENGINE_TYPE; else export GPU_BLIT_ENGINE_TYPE=$v; fi
  echo "GPU_BLIT_ENGINE_TYPE=$v" >> $o/summary.txt
  C3_EACH=6 timeout -k 10 200 python tests/tools/c3_inflight.py 6 > $o/c3_$v.txt 2> $o/c3_$v.err || { echo "rc=$?" >> $o/summary.txt; exit 1; }
  tail -1 $o/c3_$v.txt >> $o/summary.txt
done
