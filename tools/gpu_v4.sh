# k-means engine iteration: v3/v4 identity test, phase stamps (H=256), C3 bench (no CPU baseline).
export TMPDIR=/tmp
mkdir -p gpurun_out/v4
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_api.py -q -k "v4 or launch_split or seeding_cap or f64 or corr_csv" --timeout 200 --timeout-method thread > gpurun_out/v4/tests.log 2>&1; rc=$?
echo "TESTS rc=$rc"; tail -3 gpurun_out/v4/tests.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 200 python -u tools/km_stamps.py 256 > gpurun_out/v4/stamps.txt 2>&1; rc=$?; echo "STAMPS rc=$rc"; grep -v amdgpu.ids gpurun_out/v4/stamps.txt | head -14
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v4/b.json 2> gpurun_out/v4/b.err; echo "C3 rc=$?"
python -c "import json;d=json.loads(open('gpurun_out/v4/b.json').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['ms_per_step'],1), d['fit_timings_s'], {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()}, round(r['achieved'],1), round(r['frac'],4), r['sweeps'], r['slot_tile_row_tiles'])"
