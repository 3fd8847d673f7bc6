# GPU tests (fast files first, then the full-size configs) and co-association timings.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --deselect tests/test_gpu_scale.py -p no:cacheprovider > $O/tests_fast.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/tests_fast.log | tail -3; grep -E "FAILED|Error" $O/tests_fast.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/co_only.py c3 > $O/co_c3.txt 2>&1 && grep -v amdgpu.ids $O/co_c3.txt || exit 1
timeout -k 10 200 python -u tools/co_only.py c5 > $O/co_c5.txt 2>&1 && grep -v amdgpu.ids $O/co_c5.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_scale.log 2>&1
rc=$?; grep -E "passed|failed|sklearn parity|PASSED|FAILED" $O/tests_scale.log | tail -12; exit $rc
