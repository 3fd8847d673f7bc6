# sklearn parity with the engine-precision explanation: the k-means tests, the full-size C2/C4
# scale tests, and the wide engine's K=8 diagnosis.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4c; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/wide_k8_diag.py > $O/wide_k8.log 2>&1; cat $O/wide_k8.log | grep -v amdgpu
timeout -k 10 900 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_scale.py -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/scale.log 2>&1
rc=$?; grep -E "passed|failed|sklearn parity|FAILED" $O/scale.log | tail -30; exit $rc
