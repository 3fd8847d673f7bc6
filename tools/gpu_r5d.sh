# STE A/B at C3 (k-means launch alone, H = 1000, 40 GB budget) + stamps of the STE build
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d; mkdir -p $O
export KM_BUDGET_GB=40
for v in ${VARS:-prev ste}; do
  CCMI_LIB=$PWD/consensus_clustering_amd/libccmi_$v.so timeout -k 10 300 python -u tools/km_time.py ${KM_H:-1000} c3 2 > $O/km_$v.txt 2>&1 || { echo FAIL $v; tail -5 $O/km_$v.txt; exit 1; }
  grep -v amdgpu.ids $O/km_$v.txt | head -1
done
if [ -n "$STAMPS" ]; then
  KM_STAMPS_LIB=libccmi_stamps.so timeout -k 10 200 python -u tools/km_stamps.py 256 c3 > $O/st.txt 2>&1 || { echo FAIL stamps; tail -5 $O/st.txt; exit 1; }
  grep -v amdgpu.ids $O/st.txt | grep -v "n_iter per"
fi
