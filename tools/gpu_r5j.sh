# float64 engine: its GPU tests (sklearn float64 fixtures, reference float64 parity) on the
# current library, then the A/B against libccmi_f64_base.so (HEAD before the lockstep inits).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -k "f64 or float64" \
  tests/test_gpu_kmeans.py tests/test_gpu_parity_blobs.py tests/test_gpu_api.py tests/test_gpu_fit.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|f64 at|float64 input|FAILED|Error" $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
F64_CFGS="${F64_CFGS:-c3:128 c2:500 c5:64}" bash tools/gpu_f64_var.sh ${F64_VAR:-f64pk6}
