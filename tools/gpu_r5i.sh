# A/B timing (VARS) then the phase stamps of STAMP_LIBS at H=125 (one rank's share at N=8).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5i; mkdir -p $O
CFGS="${CFGS:-c3:1000 c3:125}" bash tools/gpu_r5f.sh || exit 1
for lib in ${STAMP_LIBS:-stamps}; do
  KM_STAMPS_LIB=libccmi_$lib.so timeout -k 10 200 python -u tools/km_stamps.py ${KM_H:-125} ${KM_CFG:-c3} > $O/st_$lib.txt 2>&1 || { echo stamps $lib fail; tail -3 $O/st_$lib.txt; exit 1; }
  echo "== $lib"; grep -v amdgpu.ids $O/st_$lib.txt | grep "sweeps by\|post-processing phases\|^wave [04]"
done
