#!/bin/bash
# Round 5 evidence: smoke, GPU suite, the driver's bench command, the C2 leg
# under rocprofv3 (kernel stats, MQ agreement, stream gaps), single-image
# kernel stats, PMC traffic + SQ counters (C2 leg only), MQ census.
set -o pipefail
export TMPDIR=/tmp
o=${1:-r5final}
bash tests/tools/r5_round.sh $o || exit 1
bash tests/tools/pmc_round.sh r05 || exit 1
JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/libjp2hip_debug.so timeout -k 10 200 python tests/tools/mq_census.py > gpurun_out/$o/mq_census.txt 2>&1 || exit 1
