# Parameterised GPU run (from the repo root on the box, through gpurun):
#   TAG=name               output directory gpurun_out/$TAG
#   TESTS="sel..."         pytest files/node ids run with -m gpu; unset: no tests
#   KEXPR="expr"           pytest -k expression
#   BENCH="c3 c2 ..."      bench.py configs, one JSON line each (BENCH_ARGS: extra arguments)
#   PROF=1                 rocprofv3 kernel-trace summary of `bench.py --steps 2` at the first BENCH config
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-run}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -v -s --timeout 300 --timeout-method thread -x > $OUT/tests.log 2>&1
  rc=$?
  echo "TESTS rc=$rc passed=$(grep -c ' PASSED' $OUT/tests.log)"; grep -E "FAILED|Error|error" $OUT/tests.log | head -8
  [ $rc -eq 0 ] || exit $rc
fi
for c in $BENCH; do
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py --config $c ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "BENCH_FAIL $c"; tail -5 $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);print('$c', round(d['value'],1), round(d['ms_per_step'],1), d['fit_timings_s'], {k: round(v,2) for k,v in d['kernels_ms_per_step'].items()}, 'km frac', d['roofline']['frac'], 'co frac', d['roofline_coassoc']['frac'], 'K4', d.get('roofline_consensus', {}).get('achieved'), d.get('roofline_consensus', {}).get('frac'))"
done
if [ -n "$PROF" ]; then
  c=${BENCH%% *}
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o $c --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config ${c:-c3} --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo PROF_FAIL; tail -5 $OUT/prof.log; exit 1; }
  echo PROF_OK
fi
