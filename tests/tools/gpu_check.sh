#!/bin/bash
# GPU parity suite + smoke; if green: the C2 bench line, a rocprofv3 kernel
# trace of single-image C2 encodes, and compressed-TIFF ingest timings.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-chk}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt1 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --inflight 1 --batch 1 --steps 16 > $o/bench_kt1.json 2> $o/bench_kt1.err || exit 1
timeout -k 10 300 python tests/tools/ingest_codecs.py --rps 64 --reps 2 > $o/ingest.jsonl 2> $o/ingest.err || exit 1
