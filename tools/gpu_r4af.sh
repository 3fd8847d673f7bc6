# float64 k-means against the fast engine at realistic resample counts (full C2, C3/C5 sampled)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4af; mkdir -p $O
cd $GRAFT_REPO_ROOT
for c in "c2 500" "c3 128" "c5 64"; do
  set -- $c
  timeout -k 10 400 python -u tools/f64_time.py $1 $2 2>&1 | grep -v amdgpu | tee -a $O/f64_vs_fast.txt || exit 1
done
