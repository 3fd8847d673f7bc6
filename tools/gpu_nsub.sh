# Per-rank k-means time of an 8-GPU C3 fit (rank 0 rehearsed alone) for several unit splits.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/nsub
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for ns in ${NSUBS:-2 3 4 6}; do
  CCMI_NSUB=$ns timeout -k 10 300 python -u bench.py --rehearse ${SIM:-0/8} --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b_$ns.json 2> $OUT/b_$ns.err || { echo "FAIL $ns"; tail -3 $OUT/b_$ns.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/b_$ns.json').read().strip().splitlines()[-1]);print('nsub $ns', round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()}, d['roofline']['sweeps'])"
done
