# Canonical (m, i) binning in the co-association epilogue + the batched device linkage (nn_chain
# with an LDS live mask, Prim for 'single'): tests, then C5 / C3 bench lines against
# libccmi_co_base.so (the previous co-association).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4e; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_linkage.py tests/test_gpu_coassoc.py tests/test_gpu_scale.py::test_c5_full_size tests/test_gpu_api.py -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|predict n=|single linkage n=" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for c in c5 c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
  CCMI_LIB=consensus_clustering_amd/libccmi_co_base.so timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${c}_base.json 2> $O/bench_${c}_base.err || exit $?
  python - $O/bench_$c.json $O/bench_${c}_base.json <<'PY'
import json, sys
for p in sys.argv[1:]:
    d = json.loads(open(p).read().strip().splitlines()[-1])
    print(p.split('/')[-1], 'ms/step', round(d['ms_per_step'], 1), 'coassoc', {k: round(v, 4) for k, v in d['roofline_coassoc'].items() if k in ('ms_per_fit', 'frac')}, 'kmeans ms', round(d['kernels_ms_per_step'].get('cc_kmeans_batched', 0), 1))
PY
done
