#!/bin/bash
# Round-end evidence in one call: round_final.sh (smoke, GPU suite, driver
# bench, rocprofv3 of the bench and of single-image encodes), then the C2
# bench of the previous build (libjp2hip_base.so) against this one,
# alternating, then the PMC passes (pmc_all.sh).
set -o pipefail
export TMPDIR=/tmp
r=${1:-r03}
bash tests/tools/round_final.sh ${r}_final || exit 1
o=gpurun_out/${r}_final_ab
mkdir -p $o
if [ -f jp2-bucketeer_amd/jp2hip/libjp2hip_base.so ]; then
  for i in 1 2; do
    for L in libjp2hip_base libjp2hip; do
      JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/$L.so timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-lossless > $o/b_${L}_$i.json 2> $o/b_${L}_$i.err || exit 1
      python -c "import json; d=json.loads(open('$o/b_${L}_$i.json').read().strip().splitlines()[-1]); print('$L', $i, d['value'])" | tee -a $o/summary.txt
    done
  done
fi
bash tests/tools/pmc_all.sh $r || exit 1
