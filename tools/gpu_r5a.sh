# Round 5, first GPU call: the re-pinned parity tests (sklearn fixtures), the new f64 / PAC
# tests, the linkage co-residency test, then K1 phase stamps at the C3 shape (H = 256).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_kmeans.py tests/test_gpu_parity_blobs.py tests/test_gpu_linkage.py tests/test_gpu_scale.py -k "not c4_full" \
  > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|sklearn parity|f64 at|pac_c|FAILED|Error" $O/tests.log | tail -40
case $rc in 124|137|134|139) exit $rc;; esac
if [ -n "$STAMPS" ]; then
  timeout -k 10 200 python -u tools/km_stamps.py 256 c3 > $O/stamps_c3_h256.txt 2>&1 || { echo stamps fail; tail -5 $O/stamps_c3_h256.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps_c3_h256.txt | head -20
fi
exit $rc
