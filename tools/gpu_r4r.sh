# Grid-form linkage with light barriers on the scan steps: parity tests at small n, then the
# n = 50 000 predict tests with timings (grid form, then the one-workgroup form).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4r; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py::test_manhattan_kernel_matches_scipy tests/test_gpu_linkage.py -k "oracle or manhattan or sklearn" -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/small.log 2>&1
rc=$?; grep -E "passed|failed" $O/small.log | tail -2; grep -E "^FAILED|ERROR |Error" $O/small.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_linkage.py -k "headline" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/big.log 2>&1
rc=$?; grep -E "passed|failed|predict n=|single linkage n=" $O/big.log | tail -4; grep -E "^FAILED|ERROR |Error" $O/big.log | head; [ $rc -eq 0 ] || exit $rc
CCMI_LINK_G=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_linkage.py -k "headline" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/big_g0.log 2>&1
grep -E "passed|failed|predict n=|single linkage n=" $O/big_g0.log | tail -4
