# float64 variant check: the f64 GPU tests on libccmi_$V.so, then the A/B (identity + time)
# against libccmi_f64_base.so on F64_CFGS.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5o; mkdir -p $O
CCMI_LIB=consensus_clustering_amd/libccmi_$V.so timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -k "f64 or float64" \
  tests/test_gpu_kmeans.py tests/test_gpu_parity_blobs.py tests/test_gpu_api.py tests/test_gpu_fit.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
F64_CFGS="${F64_CFGS:-c3:128 c2:500 c5:64}" bash tools/gpu_f64_var.sh $V
