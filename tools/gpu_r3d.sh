# k-means A/B at C3 (round-start library vs this build) and the phase stamps of this build.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3d; mkdir -p $O
cd $GRAFT_REPO_ROOT
LIBS="${AB_LIBS:-libccmi_base.so libccmi.so}" KM_CFG=c3 KM_REPS=2 timeout -k 10 400 bash tools/gpu_ab.sh > $O/ab_c3.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_c3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/km_stamps.py 256 c3 > $O/stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps.txt | head -16; exit $rc
