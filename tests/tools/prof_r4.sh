#!/bin/bash
# Round-4 profile of the headline configuration: the C2
# leg alone (--no-extras: no PCIe-inclusive leg, no lossless C3/C4, no C5,
# no CPU baselines), with the queue count and SDMA exported in the
# environment BEFORE rocprofv3 starts (its preload initialises the HIP
# runtime before Python runs, so bench.py's own setting would come too late),
# then the agreement of the bench's HIP-event k_t1_mq average with
# rocprofv3's average over the same launches.
set -o pipefail
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=20 JP2HIP_KEEP_HW_QUEUES=1
o=gpurun_out/${1:-prof4}
mkdir -p $o
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras > $o/bench_rocprof.json 2> $o/bench_rocprof.err || exit 1
python tests/tools/mq_agreement.py $o/bench_rocprof.json $o/kt > $o/mq_agreement.txt 2>&1 || exit 1
python tests/tools/stream_gaps.py $o/kt/run_kernel_trace.csv > $o/stream_gaps.txt 2>&1 || exit 1
python tests/tools/kstats.py $o/kt/run_kernel_stats.csv > $o/kstats.txt 2>&1 || true
