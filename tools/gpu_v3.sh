set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py -x -v --timeout 120 --timeout-method thread > gpurun_out/v3_km.log 2>&1; echo "KM rc=$?"
tail -30 gpurun_out/v3_km.log
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/v3_all.log 2>&1; echo "ALL rc=$?"
grep -E "PASS|FAIL|ERROR" gpurun_out/v3_all.log | tail -40
