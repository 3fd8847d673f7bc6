# STE A/B: the k-means launch alone at C3 (H = 1000, realistic 40 GB budget) on the HEAD build
# (prev), the STE build, and the STE build with STE sweeps off (CCMI_KM_STE=0): times and
# label / inertia / n_iter digests (identical results required).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b; mkdir -p $O
export KM_BUDGET_GB=40
for v in prev ste; do
  CCMI_LIB=$PWD/consensus_clustering_amd/libccmi_$v.so timeout -k 10 300 python -u tools/km_time.py ${KM_H:-1000} c3 2 > $O/km_$v.txt 2>&1 || { echo FAIL $v; tail -5 $O/km_$v.txt; exit 1; }
  grep -v amdgpu.ids $O/km_$v.txt
done
CCMI_KM_STE=0 CCMI_LIB=$PWD/consensus_clustering_amd/libccmi_ste.so timeout -k 10 300 python -u tools/km_time.py ${KM_H:-1000} c3 1 > $O/km_ste_off.txt 2>&1 || { echo FAIL off; exit 1; }
grep -v amdgpu.ids $O/km_ste_off.txt
