# Co-association A/B: the co-association GPU tests on the default library, then per-K timings
# (tools/co_only.py, HIP events) at each config for every library in LIBS (CCMI_LIB paths;
# "default" = consensus_clustering_amd/libccmi.so).
#   TAG=name CFGS="c3 c5 c2 c4" LIBS="default consensus_clustering_amd/libccmi_x.so" [NOTESTS=1]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-coab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_coassoc.py tests/test_gpu_parity_blobs.py -m gpu -v -s --timeout 300 --timeout-method thread -x > $OUT/tests.log 2>&1
  rc=$?
  echo "TESTS rc=$rc passed=$(grep -c ' PASSED' $OUT/tests.log)"; grep -E "FAILED|Error" $OUT/tests.log | head -8
  [ $rc -eq 0 ] || exit $rc
fi
for c in ${CFGS:-c3 c5 c2 c4}; do
  for L in ${LIBS:-default}; do
    if [ "$L" = default ]; then unset CCMI_LIB; else export CCMI_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u tools/co_only.py $c > $OUT/co_${c}_$(basename $L .so).txt 2>&1 || { echo "FAIL $c $L"; tail -3 $OUT/co_${c}_$(basename $L .so).txt; exit 1; }
    echo "$c $L: $(tail -1 $OUT/co_${c}_$(basename $L .so).txt)"
  done
done
unset CCMI_LIB
