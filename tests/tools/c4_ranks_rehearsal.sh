#!/bin/bash
# The N = 2 batch path on one GPU box: two rank processes (gloo), both on
# device 0, pulling the rows of one 96-row C4 CSV from the process group's
# store (work stealing), each through its own native queue of 12 contexts.
#   tests/tools/c4_ranks_rehearsal.sh <out-name>
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-c4ranks}
mkdir -p $o
JP2HIP_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload c4 --steps 48 --warmup 1 \
  > $o/n2.json 2> $o/n2.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --workload c4 --steps 96 --warmup 1 > $o/n1.json 2> $o/n1.err || exit 1
