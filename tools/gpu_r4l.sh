# Sparse vs dense M-step parity test (CCMI_KM_DENSE), and the C3 k-means launch with the
# diagnostic switch compiled in (kv_dflag) against the build without it (kv_base).
set -o pipefail
export TMPDIR=/tmp KM_BUDGET_GB=40
O=$GRAFT_REPO_ROOT/gpurun_out/r4l; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kmeans.py::test_sparse_mstep_against_dense -v -s --timeout 500 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|sparse vs dense|sklearn parity" $O/tests.log | tail -6; grep -E "^FAILED|ERROR |Error" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
LIBS="libccmi_kv_base.so libccmi_kv_dflag.so libccmi_kv_base.so libccmi_kv_dflag.so" KM_H=1000 KM_CFG=c3 bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu | grep -v "sweeps by active" | tee $O/kv_ab.txt
