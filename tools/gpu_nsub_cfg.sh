# k-means time at C5 / C2 for unit splits (CCMI_NSUB) and seeding-concurrency caps (CCMI_SEEDMAX).
set -o pipefail
mkdir -p gpurun_out/ns5
for v in ${VARIANTS:-NSUB=1 NSUB=2 SEEDMAX=6 SEEDMAX=16}; do
  for c in ${CFGS:-c5 c2}; do
    env CCMI_$v timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ns5/${c}_$v.json 2>/dev/null || { echo "FAIL $c $v"; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ns5/${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v', round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['kernels_ms_per_step'].items()}, d['roofline']['sweeps'])"
  done
done
