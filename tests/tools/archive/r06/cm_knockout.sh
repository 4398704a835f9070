#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r06_cmko
mkdir -p $o
for L in jp2-bucketeer_amd/jp2hip/libjp2hip.so jp2-bucketeer_amd/jp2hip/libjp2hip_cmko.so; do
  t=$(basename $L .so)
  JP2HIP_LIBRARY=$L C3_EACH=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/$t -o run --output-format csv -- python tests/tools/c3_inflight.py 1 > $o/$t.log 2>&1 || exit 1
  python3 -c "
import csv
rows=list(csv.DictReader(open('$o/$t/run_kernel_stats.csv')))
print('$t', {r['Name'].split('(')[0].replace('jp2hip::','').replace('void ','')[:14]: round(float(r['AverageNs'])/1000,1) for r in rows if float(r['AverageNs'])>50000})" | tee -a $o/summary.txt
done
