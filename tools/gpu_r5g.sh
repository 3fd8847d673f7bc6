# A/B of library variants through km_time (c3:125 = one rank's share of an N=8 C3 fit), then
# the N=8 rehearsal of bench.py for each variant.  VARS="prev lpt"
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5g; mkdir -p $O
CFGS="${CFGS:-c3:1000 c3:125 c5:256 c2:500}" VARS="${VARS:-prev lpt}" bash tools/gpu_r5f.sh || exit 1
for v in ${VARS:-prev lpt}; do
  for spec in ${SIM_SPECS:-0/8}; do
    tag=$(echo $spec | tr / _)
    CCMI_LIB=$PWD/consensus_clustering_amd/libccmi_$v.so timeout -k 10 300 python -u bench.py --rehearse $spec --steps 2 --warmup 1 --no-cpu-baseline > $O/b_${v}_$tag.json 2> $O/b_${v}_$tag.err || { echo "FAIL $v $spec"; tail -3 $O/b_${v}_$tag.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_${v}_$tag.json').read().strip().splitlines()[-1]);print('$v $spec', round(d['ms_per_step'],1), d['fit_timings_s'], {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()})"
  done
done
