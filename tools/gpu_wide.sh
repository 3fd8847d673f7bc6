# Wide-row (d > 128) k-means: GPU parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py -x -v --timeout 240 --timeout-method thread -k "wide or 300 or 2000" > gpurun_out/wide_tests.log 2>&1
rc=$?
echo "TESTS rc=$rc"
grep -E "PASSED|FAILED|ERROR|Error|assert" gpurun_out/wide_tests.log | head -30
tail -5 gpurun_out/wide_tests.log
exit $rc
