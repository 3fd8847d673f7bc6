# Phase stamps of the k-means sweep (libccmi_stamps.so, built with -DCC_KM_STAMPS).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/kmst; mkdir -p $O
for v in ${KM_STAMP_VARIANTS:-default}; do
  timeout -k 10 200 python -u tools/km_stamps.py ${KM_H:-256} ${KM_CFG:-c3} > $O/st_$v.txt 2>&1 || { echo stamps $v fail; tail -3 $O/st_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/st_$v.txt | head -16
done
