# f64 centre sums: 1, 2 or 4 feature tiles (independent MFMA chains) per wave pass, stamps builds
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ah; mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in 1 2 4; do
  echo "== FTP=$v" | tee -a $O/stamps_ftp.txt
  CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_f64ftp$v.so timeout -k 10 200 python -u tools/f64_stamps.py c3 8 c2 128 2>&1 | grep -v amdgpu | tee -a $O/stamps_ftp.txt || exit 1
done
