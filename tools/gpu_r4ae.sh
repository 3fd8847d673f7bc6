# float64 k-means: A/B of the in-tree build against libccmi_f64_base.so (tests + identity at C2/C3
# shapes, latency and throughput), then the phase split of the stamps build
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ae; mkdir -p $O
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4ad.sh || exit 1
cp gpurun_out/r4ad/* $O/
timeout -k 10 300 python -u tools/f64_stamps.py c3 8 c2 128 2>&1 | grep -v amdgpu | tee $O/stamps.txt || exit 1
