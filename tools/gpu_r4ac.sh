# float64 k-means phase split after the MFMA E-step (stamps build)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ac; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/f64_stamps.py c3 8 c2 16 c2 128 c3 48 2>&1 | grep -v amdgpu | tee $O/stamps.txt || exit 1
