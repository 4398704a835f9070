set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${1:-abround}
mkdir -p $o
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
bash tests/tools/ab_kt.sh ${1:-abround}_ab jp2-bucketeer_amd/jp2hip/libjp2hip_base.so jp2-bucketeer_amd/jp2hip/libjp2hip.so
