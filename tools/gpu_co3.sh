# co-association: tests, per-K timings (auto, exact, pow2 packing), phase stamps (diagnostic build)
export TMPDIR=/tmp
mkdir -p gpurun_out/co
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_coassoc.py -q --timeout 300 --timeout-method thread > gpurun_out/co/tests.log 2>&1; rc=$?
echo "TESTS rc=$rc"; tail -3 gpurun_out/co/tests.log
case $rc in 0) ;; *) exit $rc;; esac
fi
for pk in ${PACKS:-auto exact pow2}; do
  CCMI_CO_PACK=$pk timeout -k 10 200 python -u tools/co_only.py c3 > gpurun_out/co/c3_$pk.txt 2>&1 || exit $?
  echo "== c3 $pk"; grep -v amdgpu.ids gpurun_out/co/c3_$pk.txt | tail -2
done
CCMI_LIB=consensus_clustering_amd/libccmi_costamps.so timeout -k 10 200 python -u tools/co_stamps.py c3 ${CO_KS:-2 5 8 9 16 20} > gpurun_out/co/stamps.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/co/stamps.txt
