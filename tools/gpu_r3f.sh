# k-means A/B at C3 over library variants (AB_LIBS), then the k-means / API / fit GPU tests on
# one variant (TEST_LIB, via CCMI_LIB).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3f; mkdir -p $O
cd $GRAFT_REPO_ROOT
LIBS="$AB_LIBS" KM_CFG=${AB_CFG:-c3} KM_H=${AB_H:-1000} KM_REPS=2 timeout -k 10 500 bash tools/gpu_ab.sh > $O/ab.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.txt | grep "kmeans ms"; [ $rc -eq 0 ] || exit $rc
CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/$TEST_LIB timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_api.py tests/test_gpu_fit.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/tests.log | tail -3; grep -E "FAILED|Error|parity" $O/tests.log | head -8; exit $rc
