# Round-4 final check at HEAD: every GPU test, smoke(), the default bench line and the float64
# engine against the fast one at realistic H
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4am; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/gpu_tests.log | tail -2; grep -E "^FAILED|ERROR " $O/gpu_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo BENCH_FAIL; tail -5 $O/bench_c3.err; exit 1; }
tail -1 $O/bench_c3.json | cut -c1-250
for c in "c2 500" "c3 128" "c5 64"; do
  set -- $c
  timeout -k 10 400 python -u tools/f64_time.py $1 $2 2>&1 | grep -v amdgpu | tee -a $O/f64_vs_fast.txt || exit 1
done
