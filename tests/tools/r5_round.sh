#!/bin/bash
# Round 5 evidence set: smoke + GPU suite, the driver's bench command, the C2
# leg alone under rocprofv3 (kernel stats under load, HIP-event / rocprofv3
# agreement of k_t1_mq), and one image at a time (alone durations).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5round}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || exit 1
fi
bash tests/tools/prof_r4.sh $(basename $o)/prof || exit 1
export GPU_MAX_HW_QUEUES=8 JP2HIP_KEEP_HW_QUEUES=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-extras --inflight 1 --batch 1 --steps 12 --warmup 2 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
python tests/tools/kstats.py $o/kt1/run_kernel_stats.csv > $o/kstats_single.txt 2>&1 || true
