#!/bin/bash
# k_d2h (code-stream stores into the coherent pinned buffer, 32 workgroups)
# instead of the runtime's D2H blit: the whole GPU suite, then kernel times +
# bench vs HEAD (base), and the lossless C3 leg (PCIe-bound) of both.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r4n}
mkdir -p $o
L=jp2-bucketeer_amd/jp2hip
[ -n "$NO_SUITE" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
[ -n "$NO_SUITE" ] || tail -1 $o/t.log
AB_ROUNDS=2 bash tests/tools/ab_kt.sh ${1:-r4n}/ab $L/libjp2hip_base.so $L/libjp2hip.so || exit 1
for t in libjp2hip_base libjp2hip; do
  JP2HIP_LIBRARY=$L/$t.so timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-pcie --no-cpu-baseline > $o/full_$t.json 2> $o/full_$t.err || exit 1
  python -c "import json; d=json.loads(open('$o/full_$t.json').read().strip().splitlines()[-1]); c3=d.get('lossless_c3',{}); print('$t c2', d['value'], 'c3 inflight', c3.get('mp_per_s_inflight_c_api'), 'c3 d2h_ms', c3.get('stages_ms',{}).get('d2h_ms'), 'pcie', c3.get('roofline_pcie'))" | tee -a $o/ab/summary.txt
done
