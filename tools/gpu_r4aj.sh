# Round-4 record, part 2 (after the host-dependent parity case): the rest of gpu_r4ai.sh - the
# failed test again, the C3 bench with its CPU baseline, rocprofv3 summary, rehearsals, C2/C4/C5
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ai; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py::test_sparse_mstep_against_dense -v -s --timeout 250 --timeout-method thread -p no:cacheprovider > $O/gpu_tests_rerun.log 2>&1
rc=$?; grep -E "passed|failed|sklearn parity" $O/gpu_tests_rerun.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo BENCH_FAIL; tail -5 $O/bench_c3.err; exit 1; }
tail -1 $O/bench_c3.json | cut -c1-300
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof.log; exit 1; }
echo PROF_OK
cd $GRAFT_REPO_ROOT
for spec in 0/8 7/8 0/4 0/2; do
  tag=$(echo $spec | tr / _)
  timeout -k 10 300 python -u bench.py --rehearse $spec --steps 2 --warmup 1 --no-cpu-baseline > $O/rehearse_$tag.json 2> $O/rehearse_$tag.err || { echo "FAIL $spec"; tail -3 $O/rehearse_$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/rehearse_$tag.json').read().strip().splitlines()[-1]);print('$spec', round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()})"
done
for c in c5 c2 c4; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "FAIL $c"; tail -3 $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);print('$c', round(d['ms_per_step'],1), d['value'], d['roofline']['frac'], d.get('roofline_coassoc',{}).get('frac'))"
done
timeout -k 10 600 python -u tools/gmm_time.py 10000 16 32 > $O/gmm_time.txt 2>&1; grep -v amdgpu $O/gmm_time.txt
