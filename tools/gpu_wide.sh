# Wide-row (d > 128) k-means: GPU parity tests, then (WIDE_BENCH=1) the C4 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kmeans.py -x -v --timeout 240 --timeout-method thread -k "wide or 300 or 2000 or expression" > gpurun_out/wide_tests.log 2>&1
rc=$?
echo "TESTS rc=$rc"
grep -E "FAILED|ERROR|Error|assert" gpurun_out/wide_tests.log | head -30
tail -1 gpurun_out/wide_tests.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${WIDE_BENCH:-}" ]; then bash tools/gpu_c4.sh; fi
