#!/bin/bash
# round 4, first GPU pass: native split + sweep tests, the default bench
# (every new key), then the C2-only profile with its agreement file.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4a}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_split_native.py tests/test_gpu_sweep.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $o/t.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || exit 1
bash tests/tools/prof_r4.sh ${1:-r4a}/prof || exit 1
bash tests/tools/ab_kt.sh ${1:-r4a}/ab_ring jp2-bucketeer_amd/jp2hip/libjp2hip_ring68.so jp2-bucketeer_amd/jp2hip/libjp2hip.so || exit 1
