#!/bin/bash
# Single-image kernel times (rocprofv3 kernel stats) of several library
# builds, then the C2 bench of each:
#   tests/tools/ab_kt.sh <out-name> <lib.so> [<lib.so> ...]
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-abkt}; shift
mkdir -p $o
for L in "$@"; do
  t=$(basename $L .so)
  JP2HIP_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt_$t -o run --output-format csv -- python bench.py --no-extras --inflight 1 --batch 1 --steps 8 --warmup 2 > $o/kt_$t.json 2> $o/kt_$t.err || exit 1
  python -c "
import csv
rows=list(csv.DictReader(open('$o/kt_$t/run_kernel_stats.csv')))
print('$t', {r['Name'].split('(')[0].replace('jp2hip::','').replace('void ','')[:14]: round(float(r['AverageNs'])/1000,1) for r in rows if float(r['AverageNs'])>20000})" | tee -a $o/summary.txt
done
# the benches alternate between the builds, AB_ROUNDS times (default 2)
for r in $(seq 1 ${AB_ROUNDS:-2}); do
for L in "$@"; do
  t=$(basename $L .so)
  JP2HIP_LIBRARY=$L timeout -k 10 240 python bench.py --steps 16 --warmup 2 --no-extras > $o/b_${t}_$r.json 2> $o/b_${t}_$r.err || exit 1
  python -c "import json; d=json.loads(open('$o/b_${t}_$r.json').read().strip().splitlines()[-1]); print('$t bench $r', d['value'])" | tee -a $o/summary.txt
done
done
