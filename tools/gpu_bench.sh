set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --H 200 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v3_bench_h200.json 2> gpurun_out/v3_bench_h200.err; echo "H200 rc=$?"
cat gpurun_out/v3_bench_h200.json; tail -3 gpurun_out/v3_bench_h200.err
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v3_bench_c3.json 2> gpurun_out/v3_bench_c3.err; echo "C3 rc=$?"
cat gpurun_out/v3_bench_c3.json; tail -3 gpurun_out/v3_bench_c3.err
