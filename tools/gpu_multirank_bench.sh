# bench.py's multi-rank path (torch.distributed.run, N ranks) on a one-GPU box: every rank on
# cuda:0 over gloo (CCMI_BENCH_BACKEND=gloo; the driver's N-GPU runs use RCCL, one rank per GPU).
# Checks that the N > 1 code (barriers, max-over-ranks wall time, SUM of kernel counters and
# credited work, tile-band credit) runs and prints one JSON line.
#   SPECS="c2:2 c2:4 c3:2" bash tools/gpu_multirank_bench.sh
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/multirank
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
port=29511
for sp in ${SPECS:-c2:2 c2:4 c3:2}; do
  c=${sp%%:*}; n=${sp##*:}; port=$((port + 1))
  CCMI_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 2 --warmup 1 --config $c \
    > $OUT/${c}_n$n.json 2> $OUT/${c}_n$n.err || { echo "FAIL $sp"; tail -5 $OUT/${c}_n$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/${c}_n$n.json').read().strip().splitlines()[-1]);print('$sp', d['n_gpus'], round(d['value'],1), round(d['ms_per_step'],1), d['fit_timings_s'], 'co frac', round(d['roofline_coassoc']['frac'],3), 'partial', d['partial'])"
done
