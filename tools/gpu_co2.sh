# co-association iteration: coassoc tests, then C3 (both packings) and C5 co-association timings per K
export TMPDIR=/tmp
mkdir -p gpurun_out/co
timeout -k 10 400 python -u -m pytest tests/test_gpu_coassoc.py -q --timeout 300 --timeout-method thread > gpurun_out/co/tests.log 2>&1; rc=$?
echo "TESTS rc=$rc"; tail -5 gpurun_out/co/tests.log
case $rc in 0) ;; *) exit $rc;; esac
for pk in auto exact pow2; do
  CCMI_CO_PACK=$pk timeout -k 10 200 python -u tools/co_only.py c3 > gpurun_out/co/c3_$pk.txt 2>&1 || exit $?
  echo "== c3 $pk"; grep -v amdgpu.ids gpurun_out/co/c3_$pk.txt | tail -2
done
timeout -k 10 200 python -u tools/co_only.py c5 > gpurun_out/co/c5.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/co/c5.txt | tail -2
