#!/bin/bash
# PC sampling of the C2 bench under load (which kernels / instructions the
# resident waves sit on, with stall reasons where the method reports them).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-pcs}
mkdir -p $o
rocprofv3 -L > $o/avail.txt 2>&1 || true
grep -i -A30 "pc sampling" $o/avail.txt | head -60 > $o/pcs_configs.txt || true
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${2:-stochastic} --pc-sampling-unit ${3:-cycles} --pc-sampling-interval ${4:-1048576} --kernel-trace -d $o/run -o pcs --output-format csv -- python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-lossless > $o/bench.json 2> $o/bench.err
echo "rc=$?"
ls -R $o/run | head -20
