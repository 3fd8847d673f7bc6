export TMPDIR=/tmp
mkdir -p gpurun_out/co5
timeout -k 10 400 python -u -m pytest tests/test_gpu_coassoc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/co5/tests.log 2>&1; rc=$?
echo "TESTS rc=$rc"; tail -3 gpurun_out/co5/tests.log
[ $rc = 0 ] || exit $rc
CO_CFGS="c5 c3" CO_VARIANTS="${CO_VARIANTS:-cobase}" bash tools/gpu_co5.sh
