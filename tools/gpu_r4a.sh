# Round 4 parity checks: the n = 3000 reference fixtures (float64 and float32 input), the C2-shape
# sklearn-label injection, the tightened sklearn parity bound (k-means tests, wide engine), the
# API tests (auto precision, hybrid path over n_jobs threads, predict checks).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4a; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_blobs.py tests/test_gpu_api.py tests/test_gpu_kmeans.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1
rc=$?; grep -E "passed|failed|sklearn parity|float64 input|float32 input|C2 shape|FAILED" $O/parity.log | tail -30; exit $rc
