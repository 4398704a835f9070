#!/bin/bash
# The N-rank paths as separate processes on one GPU (gloo exchange, every
# rank on cuda:0): tile-split parts vs the single-GPU file and the oracle, the
# C2 replica bench at N=2, and the C5 tile-split bench at N=2.
set -o pipefail
export TMPDIR=/tmp JP2HIP_BENCH_BACKEND=gloo JP2HIP_BENCH_DEVICE=0
o=gpurun_out/${1:-mp}
mkdir -p $o
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
for conv in lossy lossless; do
  timeout -k 10 300 $R --master-port 29613 tests/tools/split_worker.py $o/parts_$conv $conv > $o/split_$conv.log 2>&1 || exit 1
  timeout -k 10 300 python tests/tools/split_compare.py $o/parts_$conv $conv > $o/split_$conv.json 2>> $o/split_$conv.log || exit 1
  rm -rf $o/parts_$conv
done
timeout -k 10 300 $R --master-port 29614 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline --no-lossless > $o/bench_c2_n2.json 2> $o/bench_c2_n2.err || exit 1
timeout -k 10 400 $R --master-port 29615 bench.py --gpus 2 --workload c5 --steps 2 --warmup 1 > $o/bench_c5_n2.json 2> $o/bench_c5_n2.err || exit 1
