# HEAD SQ passes (tools/gpu_sq.sh: three PMC passes each) for the co-association at C3 and C5 and
# the k-means at C3 (H = 256), after the resampling tests (the wide form is now 'auto' at C3).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4j; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_resample.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED|ERROR " $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
SQ_TAG=co_c3_r4 SQ_FILTER=tiles_kernel,-\<1, bash tools/gpu_sq.sh tools/co_only.py c3 || exit 1
SQ_TAG=co_c5_r4 SQ_FILTER=tiles_kernel,-\<1, bash tools/gpu_sq.sh tools/co_only.py c5 || exit 1
SQ_TAG=km_c3_r4 SQ_FILTER=kmeans_kernel bash tools/gpu_sq.sh tools/km_only.py 256 c3 || exit 1
