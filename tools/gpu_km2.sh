# k-means iteration: k-means GPU tests (+ full-size scale tests), then a C3 bench without the CPU baseline
export TMPDIR=/tmp
mkdir -p gpurun_out/km
timeout -k 10 600 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_scale.py tests/test_gpu_api.py tests/test_gpu_fit.py -q --timeout 300 --timeout-method thread -x > gpurun_out/km/tests.log 2>&1; rc=$?
echo "TESTS rc=$rc"; tail -6 gpurun_out/km/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/km/b.json 2> gpurun_out/km/b.err; echo "C3 rc=$?"
python -c "import json;d=json.loads(open('gpurun_out/km/b.json').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['ms_per_step'],1), d['fit_timings_s'], {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()}, round(r['achieved'],1), round(r['frac'],4), r['sweeps'], r['slot_tile_row_tiles'])"
