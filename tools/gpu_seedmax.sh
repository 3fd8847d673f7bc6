# C3 k-means time for several concurrent-seeding limits (CCMI_SEEDMAX).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/sm
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for sm in ${SMS:-8 16 24 32}; do
  CCMI_SEEDMAX=$sm timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/b_$sm.json 2> $OUT/b_$sm.err || { echo "FAIL $sm"; tail -3 $OUT/b_$sm.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b_$sm.json').read().strip().splitlines()[-1]);print('seedmax $sm', round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()}, d['roofline']['sweeps'])"
done
