set -o pipefail
mkdir -p gpurun_out/sw
for n in 12 16 24 28; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-lossless --steps 96 --inflight $n > gpurun_out/sw/if$n.json 2> gpurun_out/sw/if$n.err || exit 1
done
