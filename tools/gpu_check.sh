set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r01_gpu_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u bench.py > gpurun_out/r01_bench.json 2> gpurun_out/r01_bench.err && echo BENCH_OK && cat gpurun_out/r01_bench.json
