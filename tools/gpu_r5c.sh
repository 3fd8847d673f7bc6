# Phase stamps of the HEAD and STE builds at the C3 shape (H = 256)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c; mkdir -p $O
for v in stampsprev stamps; do
  KM_STAMPS_LIB=libccmi_$v.so timeout -k 10 200 python -u tools/km_stamps.py 256 c3 > $O/st_$v.txt 2>&1 || { echo FAIL $v; tail -5 $O/st_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/st_$v.txt | grep -v "n_iter per"
done
