#!/bin/bash
# C3 in flight with the code-stream D2H left out (diagnostic build): is the
# in-flight rate bound by the GPU's work or by the PCIe copy?
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3n}
mkdir -p $o
JP2HIP_LIBRARY=jp2-bucketeer_amd/jp2hip/libjp2hip_nod2h.so timeout -k 10 300 python tests/tools/c3_inflight.py 4 6 8 > $o/nod2h.json 2> $o/nod2h.err || exit 1
timeout -k 10 300 python tests/tools/c3_inflight.py 4 6 8 > $o/product.json 2> $o/product.err || exit 1
