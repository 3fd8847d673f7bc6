# Round record: full GPU tests, the C3 bench (with CPU baseline), a rocprofv3 kernel-trace
# summary of the bench, and the HBM-traffic PMC passes of the k-means launch (FETCH_SIZE and
# WRITE_SIZE in separate passes).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/rec
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "TESTS rc=$rc"; grep -cE "PASSED" $OUT/gpu_tests.log; grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -5 $OUT/bench.err; exit 1; }
echo BENCH_OK; tail -1 $OUT/bench.json | cut -c1-400
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo PROF_FAIL; tail -5 $OUT/prof.log; exit 1; }
echo PROF_OK
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/km_only.py 1000 > $OUT/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; tail -3 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/km_only.py 1000 > $OUT/pmc_write.log 2>&1 || { echo PMC2_FAIL; tail -3 $OUT/pmc_write.log; exit 1; }
echo PMC_OK
for spec in ${SIM_SPECS:-0/8 7/8}; do
  tag=$(echo $spec | tr / _)
  timeout -k 10 300 python -u $GRAFT_REPO_ROOT/bench.py --rehearse $spec > $OUT/rehearse_$tag.json 2> $OUT/rehearse_$tag.err || { echo "REHEARSE_FAIL $spec"; tail -3 $OUT/rehearse_$tag.err; exit 1; }
  echo "REHEARSE $spec $(tail -1 $OUT/rehearse_$tag.json | cut -c1-300)"
done
