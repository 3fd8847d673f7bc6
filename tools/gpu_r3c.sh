# Sparse M-step check: k-means launch A/B (round-start library vs this build) at C3 and C5,
# then the k-means / API / fit GPU tests on this build.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3c; mkdir -p $O
cd $GRAFT_REPO_ROOT
LIBS="libccmi_base.so libccmi.so" KM_CFG=c3 KM_REPS=2 timeout -k 10 400 bash tools/gpu_ab.sh > $O/ab_c3.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_c3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_api.py tests/test_gpu_fit.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/tests.log | tail -3; grep -E "FAILED|Error|parity" $O/tests.log | head -8; [ $rc -eq 0 ] || exit $rc
LIBS="libccmi_base.so libccmi.so" KM_CFG=c5 KM_H=256 KM_REPS=2 timeout -k 10 300 bash tools/gpu_ab.sh > $O/ab_c5.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_c5.txt; exit $rc
