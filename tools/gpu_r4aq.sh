# Round-4 last check at HEAD: every GPU test and smoke()
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4aq; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/gpu_tests.log | tail -2; grep -E "^FAILED|ERROR " $O/gpu_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
