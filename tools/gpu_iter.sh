set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_tests.log 2>&1; echo "TESTS rc=$?"; tail -3 gpurun_out/it_tests.log
timeout -k 10 200 python -u tools/km_stamps.py 256 > gpurun_out/it_stamps.txt 2>&1; echo "STAMPS rc=$?"; grep -v amdgpu.ids gpurun_out/it_stamps.txt | head -14
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/it_bench.json 2> gpurun_out/it_bench.err; echo "C3 rc=$?"
python -c "import json;d=json.load(open('gpurun_out/it_bench.json'));print(d['ms_per_step'], d['fit_timings_s'], d['kernels_ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])"
