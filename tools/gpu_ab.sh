set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; echo "TESTS(owned) rc=$?"; tail -2 gpurun_out/ab_tests.log
CCMI_KM_SHARED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests2.log 2>&1; echo "TESTS(shared) rc=$?"; tail -2 gpurun_out/ab_tests2.log
for mode in owned shared; do
  if [ $mode = shared ]; then export CCMI_KM_SHARED=1; fi
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || { echo "bench $mode failed"; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_$mode.json').read().splitlines()[-1]);print('$mode', d['ms_per_step'], d['kernels_ms_per_step']['cc_kmeans_batched'], d['roofline']['sweeps'], d['roofline']['slot_tile_row_tiles'])"
done
