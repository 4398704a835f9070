#!/bin/bash
# Do the code-stream D2H copies run as blit kernels with HSA_ENABLE_SDMA
# unset / 0 / 1?  (rocprofv3 kernel trace of a short C2-only bench each)
set -o pipefail
export TMPDIR=/tmp JP2HIP_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=20
o=gpurun_out/${1:-sdma_probe}
mkdir -p $o
for v in unset 0 1; do
  if [ $v = unset ]; then unset HSA_ENABLE_SDMA; else export HSA_ENABLE_SDMA=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt_$v -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-extras > $o/b_$v.json 2> $o/b_$v.err || exit 1
  echo "SDMA=$v: $(grep -c copyBuffer $o/kt_$v/run_kernel_trace.csv) copyBuffer dispatches, value $(python -c "import json;print(json.loads(open('$o/b_$v.json').read().strip().splitlines()[-1])['value'])")" | tee -a $o/summary.txt
done
