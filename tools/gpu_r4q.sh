# Linkage grid size sweep at n = 50 000 (CCMI_LINK_G), headline predict tests, timings only.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4q; mkdir -p $O
cd $GRAFT_REPO_ROOT
for g in 16 64 128 32; do
  CCMI_LINK_G=$g timeout -k 10 300 python -u -m pytest tests/test_gpu_linkage.py -k "headline" -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/g$g.log 2>&1 || { echo "FAIL G=$g"; tail -5 $O/g$g.log; exit 1; }
  echo "G=$g: $(grep -E 'predict n=|single linkage n=' $O/g$g.log | tr '\n' ' ')"
done
