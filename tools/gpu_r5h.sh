# Phase stamps: one rank's share of an N=8 C3 fit (H=125), workgroup 0 then the narrow
# (<= 32 slot) sweeps of every workgroup; then the N=1 fit (H=1000), workgroup 0.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h; mkdir -p $O
for spec in stamps:125 stampsn:125 stamps:1000; do
  lib=${spec%%:*}; H=${spec##*:}
  KM_STAMPS_LIB=libccmi_$lib.so timeout -k 10 200 python -u tools/km_stamps.py $H ${KM_CFG:-c3} > $O/st_${lib}_$H.txt 2>&1 || { echo stamps $lib fail; tail -3 $O/st_${lib}_$H.txt; exit 1; }
  echo "== $lib $H"; grep -v amdgpu.ids $O/st_${lib}_$H.txt
done
