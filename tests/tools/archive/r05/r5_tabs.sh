#!/bin/bash
# MQ next-state table copies (1 / 2 / 4): parity, single-image stage times,
# k_t1_mq LDS bank conflicts (PMC), C2 bench A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5tabs}
L=jp2-bucketeer_amd/jp2hip
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/parity.txt 2>&1 || exit 1
for V in libjp2hip libjp2hip_tab1 libjp2hip_tab4; do
  JP2HIP_LIBRARY=$L/$V.so timeout -k 10 200 python tests/tools/mq_alone.py > $o/alone_$V.txt 2>&1 || exit 1
  JP2HIP_LIBRARY=$L/$V.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU --kernel-include-regex "k_t1_mq" -d $o/pmc_$V -o run --output-format csv -- python tests/tools/mq_alone.py > $o/pmc_$V.log 2>&1 || exit 1
done
bash tests/tools/ab_lib.sh $(basename $o)/ab $L/libjp2hip.so $L/libjp2hip_tab1.so 2 || exit 1
