set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ext; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_coassoc.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c5 c3 c2 c4; do
  for L in default cobase; do
    if [ $L = default ]; then unset CCMI_LIB; else export CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_cobase.so; fi
    timeout -k 10 300 python -u bench.py --config $c --steps 3 --no-cpu-baseline --no-consensus-roofline > $O/b_${c}_$L.json 2>$O/b_${c}_$L.err || { echo "FAIL $c $L"; tail -3 $O/b_${c}_$L.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_${c}_$L.json').read().strip().splitlines()[-1]);k=d['kernels_ms_per_step'];print('$c $L band', round(k['coassoc_band'],2), 'launch_sum', round(k['cc_coassoc'],2), 'frac', round(d['roofline_coassoc']['frac'],4), 'ms', round(d['ms_per_step'],1))"
  done
done
unset CCMI_LIB
for c in c5 c3; do
  for L in default cobase; do
    if [ $L = default ]; then unset CCMI_LIB; else export CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_cobase.so; fi
    timeout -k 10 300 python -u tools/co_only.py $c > $O/co_${c}_$L.txt 2>&1 || { echo "FAIL co $c $L"; exit 1; }
    echo "uniform-labels $c $L: $(tail -1 $O/co_${c}_$L.txt)"
  done
done
