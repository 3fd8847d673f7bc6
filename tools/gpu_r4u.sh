# Parity census of the f32-class k-means on C3-shaped blobs, 8 data seeds.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4u; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u tools/parity_census.py 4000 4 2 8 9 2>&1 | grep -v amdgpu | tee $O/census.txt
