#!/bin/bash
# The committed tree as the driver runs it at round end: smoke, the GPU
# suite, the driver's bench command (every leg), then the footprint records.
#   tests/tools/final_check.sh <out-name>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-final_check}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 800 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 python -u tests/tools/footprint.py $o/footprint.jsonl > $o/footprint.log 2>&1 || exit 1
