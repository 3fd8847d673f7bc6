# C2 and C5 bench lines (no CPU baseline) for the DESIGN config table.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/cfg
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for c in ${CFGS:-c2 c5}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$c.json 2> $OUT/$c.err || { echo "FAIL $c"; tail -3 $OUT/$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/$c.json').read().strip().splitlines()[-1]);print('$c', round(d['ms_per_step'],1), d['fit_timings_s'], {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()})"
done
