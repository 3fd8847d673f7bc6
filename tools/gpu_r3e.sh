# k-means A/B at C3 (round-start library vs this build), phase stamps of this build, k-means tests.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3e; mkdir -p $O
cd $GRAFT_REPO_ROOT
LIBS="${AB_LIBS:-libccmi_base.so libccmi.so}" KM_CFG=${AB_CFG:-c3} KM_H=${AB_H:-1000} KM_REPS=2 timeout -k 10 400 bash tools/gpu_ab.sh > $O/ab.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/km_stamps.py 256 c3 > $O/stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps.txt | head -16; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_api.py tests/test_gpu_fit.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/tests.log | tail -3; grep -E "FAILED|Error|parity" $O/tests.log | head -8; exit $rc
