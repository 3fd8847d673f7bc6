# C4 (n=5k, d=20k, K=2..12, H=1000) bench + rocprof kernel stats of a shorter run.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/c4
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py --config c4 --steps 1 --warmup 1 ${C4_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -5 $OUT/bench.err; exit 1; }
echo BENCH_OK
python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['fit_timings_s'], d['kernels_ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['sweeps'], d.get('cpu_baseline',{}).get('value'))"
if [ -n "${C4_PROF:-}" ]; then
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 1 --warmup 0 --H 200 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo PROF_FAIL; tail -5 $OUT/prof.log; exit 1; }
echo PROF_OK
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 > $OUT/stats_short.csv; cut -c1-160 $OUT/stats_short.csv | tail -n +1 | sed -n 1,8p
fi
