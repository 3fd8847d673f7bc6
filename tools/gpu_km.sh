# k-means change check: GPU k-means + API tests, then the C3 bench (no CPU baseline).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/km
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 $OUT/tests.log; grep -E "^FAILED|Error" $OUT/tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline ${KM_ARGS:-} > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAIL; tail -3 $OUT/b.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],1), d['fit_timings_s'], {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()}, round(d['roofline']['achieved'],1), d['roofline']['sweeps'])"
