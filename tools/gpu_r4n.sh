# Co-association bin table copied by LDS-DMA with every piece in flight: its exactness tests,
# then C5 / C3 / C2 benches against the base build, same box.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4n; mkdir -p $O
cd $GRAFT_REPO_ROOT
CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_co_dma.so timeout -k 10 600 python -u -m pytest tests/test_gpu_coassoc.py tests/test_gpu_parity_blobs.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED|ERROR " $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
for c in c5 c3 c2; do
  for lib in co_base co_dma co_base co_dma; do
    CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_$lib.so timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_${c}_$lib.json 2> $O/bench_${c}_$lib.err || { echo "FAIL $c $lib"; tail -3 $O/bench_${c}_$lib.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/bench_${c}_$lib.json').read().strip().splitlines()[-1]);r=d['roofline_coassoc'];print('$c $lib', round(d['ms_per_step'],1), 'co ms', round(r['ms_per_fit'],2), 'sum', round(r.get('launch_ms_sum_per_fit',0),2), 'frac', round(r['frac'],3))"
  done
done
