# Per-K co-association launches over side streams (engine.coassoc_all): parity tests, then the
# C2/C4/C5/C3 benches with 1 / 2 / 3 streams; the process-pool host fits with one BLAS thread.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4h; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_coassoc.py tests/test_gpu_api.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED|ERROR " $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
for c in c2 c4 c5 c3; do
  for s in 1 2 3; do
    CCMI_CO_STREAMS=$s timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${c}_s$s.json 2> $O/bench_${c}_s$s.err || { echo "FAIL $c $s"; tail -3 $O/bench_${c}_s$s.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/bench_${c}_s$s.json').read().strip().splitlines()[-1]);r=d['roofline_coassoc'];print('$c streams $s', round(d['ms_per_step'],1), 'co ms', round(r['ms_per_fit'],2), 'sum', round(r.get('launch_ms_sum_per_fit',0),2), 'frac', round(r['frac'],3), 'issued', round(r.get('frac_of_issued_instruction_peak',0),3))"
  done
done
timeout -k 10 600 python -u tools/gmm_time.py 10000 16 32 > $O/gmm_time.txt 2>&1; grep -v amdgpu $O/gmm_time.txt
