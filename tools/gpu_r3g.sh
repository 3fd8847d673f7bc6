# predict(): device linkage tests (oracle equality, n = 50k), the API tests (golden consensus
# labels through the device path), and the full-size scale tests (sklearn parity).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3g; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_linkage.py tests/test_gpu_api.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/linkage.log 2>&1
rc=$?; grep -E "passed|failed|error|predict n=" $O/linkage.log | tail -5; grep -E "FAILED|Error" $O/linkage.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/scale.log 2>&1
rc=$?; grep -E "passed|failed|sklearn parity|FAILED" $O/scale.log | tail -8; exit $rc
