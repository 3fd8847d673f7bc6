# float64 k-means: the MFMA f64 rounding probe, the batched serial loads A/B (identity vs the
# committed kernel), and the stamps split at latency (few units) and throughput (many units) shapes.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ab; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/mfma_f64_probe | tee $O/probe.txt || exit 1
bash tools/gpu_r4aa.sh || exit 1
cp gpurun_out/r4aa/* $O/ 2>/dev/null
timeout -k 10 500 python -u tools/f64_stamps.py c3 8 c2 16 c2 128 c3 48 2>&1 | grep -v amdgpu | tee $O/stamps.txt || exit 1
