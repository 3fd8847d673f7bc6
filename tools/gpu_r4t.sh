# Where the C3 k-means launch spends its time by phase: max_iter = 1 / 2 / 5 / 300 (k-means++
# seeding plus that many Lloyd iterations; timing only, the labels are not the fit's).
set -o pipefail
export TMPDIR=/tmp KM_BUDGET_GB=40
O=$GRAFT_REPO_ROOT/gpurun_out/r4t; mkdir -p $O
cd $GRAFT_REPO_ROOT
for it in 1 2 5 300; do
  KM_MAXITER=$it timeout -k 10 300 python -u tools/km_time.py 1000 c3 1 2>&1 | grep -v amdgpu | grep -v "sweeps by active" | sed "s/^/max_iter=$it: /" | tee -a $O/phase.txt || exit 1
done
