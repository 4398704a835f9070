#!/bin/bash
# D2H copy engine under different runtime settings (tests/tools/d2h_engine_probe.py)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-d2hprobe}
mkdir -p $o
i=0
for e in "X=1" "HSA_ENABLE_SDMA=1" "ROC_ENABLE_LARGE_BAR=0" "GPU_FORCE_BLIT_COPY_SIZE=0" "HSA_FORCE_SDMA_SIZE=1" \
         "ROC_ENABLE_LARGE_BAR=0 HSA_ENABLE_SDMA=1" "GPU_BLIT_ENGINE_TYPE=1" "GPU_CP_DMA_COPY_SIZE=1"; do
  i=$((i+1))
  env $e timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $o/p$i -o run --output-format csv -- python tests/tools/d2h_engine_probe.py > $o/p$i.log 2>&1 || { echo "fail $e"; exit 1; }
  n=$(grep -c copyBuffer $o/p$i/*/run_kernel_trace.csv 2>/dev/null || grep -c copyBuffer $o/p$i/run_kernel_trace.csv 2>/dev/null || echo 0)
  echo "$e -> copyBuffer dispatches: $n; $(grep GBps $o/p$i.log)" | tee -a $o/summary.txt
done
