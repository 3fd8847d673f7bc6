# Rehearse the per-rank critical path of an N-GPU C3 fit on one GPU (bench.py --rehearse r/N).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/sim
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for spec in ${SIM_SPECS:-0/8 7/8 0/4 0/2}; do
  tag=$(echo $spec | tr / _)
  timeout -k 10 300 python -u bench.py --rehearse $spec --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "FAIL $spec"; tail -3 $OUT/b_$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b_$tag.json').read().strip().splitlines()[-1]);print('$spec', round(d['ms_per_step'],1), d['fit_timings_s'], {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()})"
done
