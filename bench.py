"""Consensus-fit benchmark (BASELINE.json metric) on 1..N MI355X GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One STEP is one full ``ConsensusClustering.fit`` of the workload (all K, all H
resamples: resampling, batched k-means, co-sampling, co-association + histogram,
host CDF/PAC), with X already resident in HBM.  Default workload = BASELINE config 3
(the metric's own: synthetic blobs n=50k, d=128, K=2..20, H=1000, subsampling 0.8),
strong scaling: the ranks split the fixed fit (resamples for k-means, triangle tiles
for co-association).  Rank 0 prints ONE JSON line.

``roofline`` is the dominant kernel (cc_kmeans_batched, MFMA-bound): ALGORITHMIC flops
FLOP_KM of SURVEY.md §8d (2·d per row×centroid distance product of Lloyd and k-means++; the
kernel counts the products) ÷ the launches' HIP-event durations on the launch stream, against
the f32-class ceiling of the f16 hi/lo MFMA scheme (2516.6 TF f16 dense / 3 = 838.9 TF).  The
M-step's d flops per (row, running problem) update are not part of §8d's FLOP_KM; they are
reported beside it (``mstep_flops_per_launch``, ``frac_incl_mstep``).  A fraction above 1
means the timed launches did not do the credited work: the bench refuses to report it.
``cpu_baseline`` times the oracle (numpy + scikit-learn, the reference's algorithm) on a
bounded sample of the same workload on this host's usable cores and extrapolates to
resample-clusterings/s (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as tdist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "consensus fit wall-time + resample-clusterings/sec, n=50k d=128, 1/2/4/8 GPU"
CONFIGS = {
    # BASELINE.json configs[2]: the metric's workload
    "c3": dict(n=50_000, d=128, k_true=8, Ks=list(range(2, 21)), H=1000, frac=0.8),
    # BASELINE.json configs[1] / configs[4], for ad-hoc runs
    "c2": dict(n=10_000, d=64, k_true=6, Ks=list(range(2, 16)), H=500, frac=0.8),
    "c5": dict(n=200_000, d=32, k_true=6, Ks=list(range(2, 11)), H=256, frac=0.8),
    # BASELINE.json configs[3]: wide rows (cc_kmeans_wide)
    "c4": dict(n=5_000, d=20_000, k_true=5, Ks=list(range(2, 13)), H=1000, frac=0.8,
               data="expression"),
    "smoke": dict(n=4_000, d=32, k_true=5, Ks=list(range(2, 8)), H=64, frac=0.8),
}
# MI355X_MICROARCH.md: f16/bf16 dense MFMA peak 256 CU x 4 SIMD x 1024 flop/clk x 2.4 GHz.  One
# f32-class product costs three f16 MFMA products (xh.ch + xh.cl + xl.ch), so the ceiling for
# the algorithmic (f32-equivalent) flops of the k-means is a third of it.
F16_MFMA_PEAK_TF = 2516.6
KMEANS_PEAK_TF = F16_MFMA_PEAK_TF / 3
I8_MFMA_PEAK_TOPS = 2 * F16_MFMA_PEAK_TF  # v_mfma_i32_32x32x32_i8: 2x the f16 rate
FP4_MFMA_PEAK_TOPS = 4 * F16_MFMA_PEAK_TF  # v_mfma_scale_f32_32x32x64_f8f6f4, e2m1: 4x the f16 rate
SEED = 0


def make_blobs_f32(n, d, k, seed=0):
    """sklearn.datasets.make_blobs(n, d, centers=k, cluster_std=1, center_box=(-10, 10),
    shuffle=True, random_state=seed) cast to float32."""
    from sklearn.datasets import make_blobs

    X, _ = make_blobs(n_samples=n, n_features=d, centers=k, cluster_std=1.0,
                      center_box=(-10.0, 10.0), shuffle=True, random_state=seed)
    return X.astype(np.float32)


def make_expression_f32(n, d, groups=5, informative=500, shift_std=2.0, seed=0):
    """BASELINE config 4's gene-expression-like rows: n samples in `groups`
    groups; the first `informative` features carry a per-group mean shift ~ N(0, shift_std^2),
    every feature has N(0, 1) noise; float32."""
    rs = np.random.RandomState(seed)
    g = rs.randint(0, groups, size=n)
    means = np.zeros((groups, d), dtype=np.float32)
    means[:, :informative] = rs.normal(0.0, shift_std, size=(groups, informative))
    X = rs.standard_normal((n, d)).astype(np.float32)
    X += means[g]
    return X


def _timed_fit(X, idx_row, K):
    """One reference fit (CC.py:282, sklearn KMeans n_init=3) on one BLAS/OpenMP thread."""
    from threadpoolctl import threadpool_limits

    from oracle import cc_oracle as O

    with threadpool_limits(1):
        t = time.perf_counter()
        lab = O.kmeans_labels(X[idx_row], K, SEED, n_init=3)
        return time.perf_counter() - t, lab


def _timed_coassoc(n, idx_row, lab, K, block):
    """CC.py:284-290 for one (h, K) on a `block`-row slice of the n x n uint16 M: one-hot L of
    that fit's own labels, the integer L^T L and the in-place add (one thread)."""
    from threadpoolctl import threadpool_limits

    with threadpool_limits(1):
        L = np.zeros((K, n), dtype=np.uint16)
        L[lab, idx_row] = 1
        Mblk = np.zeros((block, n), dtype=np.uint16)
        t = time.perf_counter()
        Mblk += np.dot(L[:, :block].T, L)
        return time.perf_counter() - t


def cpu_baseline(cfg, X, H_sample=8):
    """The reference's parallelised CPU path (CC.py:162-199, joblib processes, n_jobs = the
    box's CPU share) timed on a bounded sample of the same workload and
    extrapolated linearly in H:

      T = T_I(H) + Σ_K [H / H' · T_fits(K, H')] + Σ_K H · t_co(K) / n_jobs + Σ_K t_an(K)

    * T_fits: all K, H' resamples, every KMeans fit a joblib process task with one BLAS thread;
    * t_co(K): one (h, K) co-association (one-hot L^T L + in-place add, CC.py:284-290) timed on
      a row block and scaled to n rows, for 3 sampled K and interpolated (the reference runs
      these inside the same n_jobs workers);
    * T_I: the integer S^T S (CC.py:264) and t_an: C = M / I + histogram (CC.py:338-373), both
      serial in the reference, timed on row blocks and scaled to n rows.
    """
    from joblib import Parallel, delayed
    from threadpoolctl import threadpool_limits

    from oracle import cc_oracle as O

    n, H, frac = cfg["n"], cfg["H"], cfg["frac"]
    Ks = cfg["Ks"]
    cores = usable_cores()
    Hs = min(H, H_sample)
    idx = O.subsampling_indices(n, Hs, frac, SEED)
    t0 = time.perf_counter()
    print(f"[bench] cpu baseline: {cores} joblib processes", file=sys.stderr, flush=True)
    with Parallel(n_jobs=cores, prefer="processes") as par:
        a = time.perf_counter()
        fits = par(delayed(_timed_fit)(X, idx[h], K) for K in Ks for h in range(Hs))
        T_fits = (time.perf_counter() - a) * (H / Hs)
        print("[bench] cpu baseline: fits sampled", file=sys.stderr, flush=True)
        block = min(n, 1000)
        sampleK = sorted({Ks[0], Ks[len(Ks) // 2], Ks[-1]})
        lab0 = {K: fits[k * Hs][1] for k, K in enumerate(Ks)}  # resample 0's labels of each K
        tco = par(delayed(_timed_coassoc)(n, idx[0], lab0[K], K, block) for K in sampleK)
    t_co = {K: t * (n / block) for K, t in zip(sampleK, tco)}
    T_co = sum(H * np.interp(K, sampleK, [t_co[k] for k in sampleK]) for K in Ks) / cores
    # I = S^T S (serial numpy integer matmul) and the per-K analysis, on row blocks
    with threadpool_limits(1):
        bI = min(n, 200)
        S = (np.random.RandomState(0).rand(H, n) < frac).astype(np.uint16 if H >= 256 else np.uint8)
        a = time.perf_counter()
        np.dot(S[:, :bI].T, S)
        T_I = (time.perf_counter() - a) * (n / bI)
        print("[bench] cpu baseline: S^T S sampled", file=sys.stderr, flush=True)
        bA = min(n, 500)
        M = np.random.RandomState(1).randint(0, H + 1, size=(bA, n), dtype=S.dtype)
        I = np.maximum(M, H // 2).astype(S.dtype)
        a = time.perf_counter()
        C = np.divide(M, I + 1e-6, dtype=np.float32)
        np.histogram(np.triu(C, k=1).ravel(), bins=20, range=(0, 1), density=True)
        T_an = (time.perf_counter() - a) * (n / bA) * len(Ks)
    total = T_I + T_fits + T_co + T_an
    return {
        "value": H * len(Ks) / total,
        "unit": "resample-clusterings/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"reference algorithm (oracle: numpy {np.__version__} + sklearn "
                   f"{__import__('sklearn').__version__} KMeans n_init=3), joblib processes "
                   f"n_jobs={cores} x 1 BLAS thread (CC.py:185-195): all {len(Ks)} K x H'={Hs} "
                   f"resample fits timed ({T_fits * Hs / H:.1f} s wall), extrapolated x{H / Hs:.0f} "
                   f"in H; co-association L^T L + add (the sampled fits' own labels) timed on a "
                   f"{block}-row block for K in {sampleK} and scaled to n rows / n_jobs; S^T S ({bI}-row block) and "
                   f"C/histogram ({bA}-row block) serial, scaled to n rows. Extrapolated fit "
                   f"{total / 3600:.2f} h = I {T_I:.0f} s + fits {T_fits:.0f} s + co-association "
                   f"{T_co:.0f} s + analysis {T_an:.0f} s; sampled {time.perf_counter() - t0:.1f} s"),
    }


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured float4 copy)


def consensus_roofline(dev, n, H, reps=5):
    """cc_consensus (K4, CC.py:372-373: C = f32(M) / f32(I + 1e-6), diag 1) on n x n int32 M and I
    resident in HBM, the pass that runs whenever cij or predict is asked for: 12 algorithmic bytes
    per element (two int32 reads, one float32 write) / the average launch time (HIP events on the
    launch stream), against the 8 TB/s HBM peak.  Measured after the timed fits, outside them."""
    from consensus_clustering_amd import engine

    g = torch.Generator(device=dev)
    g.manual_seed(0)
    I = torch.randint(H // 2, H + 1, (n, n), dtype=torch.int32, device=dev, generator=g)
    M = torch.randint(0, H // 2 + 1, (n, n), dtype=torch.int32, device=dev, generator=g)  # M <= I
    engine.consensus(M, I)  # warm-up (and the allocation of C)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        C = engine.consensus(M, I)
        b.record()
        del C
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in evs) / reps
    nbytes = 12.0 * n * n
    achieved = nbytes / (ms * 1e-3) / 1e9
    del M, I
    torch.cuda.empty_cache()
    return {"kernel": "cc_consensus", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": checked_frac(achieved, HBM_PEAK_GBS, "consensus"),
            "traffic": None, "n": n, "bytes_per_launch": nbytes, "avg_launch_ms": ms,
            "note": "K4 C = M / (I + 1e-6) over n x n int32 M, I (12 B per element); runs when "
                    "keep_matrices or predict asks for C, not inside the timed fit"}


def usable_cores() -> int:
    """CPUs this process may use: its affinity mask, capped by the cgroup CPU quota (a GPU box
    shows every host CPU in the mask but grants one GPU's share of them)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        n = os.cpu_count() or 1
    quota = None
    try:  # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return n


def band_pairs(n: int, tile_begin: int, tile_end: int, T: int = 256) -> int:
    """Strict-upper pairs (i < j < n) inside the upper-triangle tiles [tile_begin, tile_end),
    numbered row-major as cc_coassoc numbers them (tile (bi, bj), bi <= bj)."""
    nb = (n + T - 1) // T
    total, t = 0, 0
    for bi in range(nb):
        row_tiles = nb - bi
        lo, hi = max(tile_begin, t), min(tile_end, t + row_tiles)
        if lo < hi:
            rows = min(n, (bi + 1) * T) - bi * T
            for bj in range(bi + (lo - t), bi + (hi - t)):
                if bj == bi:
                    total += rows * (rows - 1) // 2
                else:
                    total += rows * (min(n, (bj + 1) * T) - bj * T)
        t += row_tiles
    return total


def checked_frac(achieved, peak, what):
    """achieved / peak, or None (with a note on stderr) when it exceeds 1: a fraction above the
    roof means the timed launches did not do the credited work."""
    if peak <= 0:
        return None
    f = achieved / peak
    if f > 1.0:
        print(f"[bench] REFUSED: {what} roofline fraction {f:.3f} > 1 (credited work was not all "
              "done by the timed launches)", file=sys.stderr, flush=True)
        return None
    return f


def load_traffic(config, kernel, key="bytes_per_launch", prefix="profiles"):
    """HBM bytes of `kernel` at `config` (per launch, or per fit with key="bytes_per_fit") from a
    committed PMC summary (profiles/traffic/<config>_<kernel>.json, tools/traffic_summary.py), or
    None when no such measurement exists."""
    path = os.path.join(ROOT, prefix, "traffic", f"{config}_{kernel}.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f).get(key)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-consensus-roofline", action="store_true")
    ap.add_argument("--H", type=int, default=None, help="override n_iterations (debug runs)")
    ap.add_argument("--rehearse", default=None, metavar="R/N",
                    help="one-GPU rehearsal of rank R's share of an N-GPU fit (exchanges skipped; "
                         "the fit's results are partial, the timing is rank R's critical path)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.H:
        cfg["H"] = args.H

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # CCMI_BENCH_BACKEND=gloo (tests only): every rank on device LOCAL_RANK mod the device count
        # over gloo, to exercise this multi-rank path on a one-GPU box, where RCCL refuses two ranks
        # on one device; the driver's N-GPU runs use RCCL ("nccl"), one rank per GPU
        backend = os.environ.get("CCMI_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            tdist.init_process_group(backend)
    dev = torch.device("cuda", torch.cuda.current_device())

    from consensus_clustering_amd import ConsensusClustering, engine
    from consensus_clustering_amd.dist import shard as dist_shard

    if cfg.get("data") == "expression":
        X = make_expression_f32(cfg["n"], cfg["d"], groups=cfg["k_true"], seed=SEED)
        data = "synthetic gene-expression-like (5 groups, 500 informative features, N(0,1) noise, float32, seed 0)"
    else:
        X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"], seed=SEED)
        data = "synthetic (make_blobs, float32, seed 0)"
    Xd = torch.from_numpy(X).to(dev)  # inputs resident in HBM before the timed region
    cc = ConsensusClustering(K_range=cfg["Ks"], n_iterations=cfg["H"], subsampling=cfg["frac"],
                             random_state=SEED, plot_cdf=False, keep_matrices=False)
    if args.rehearse:
        r, w = (int(v) for v in args.rehearse.split("/"))
        cc._rehearsal = (r, w)

    def barrier():
        if world > 1:
            tdist.barrier()

    for i in range(args.warmup):
        cc.fit(Xd)
        print(f"[bench] warmup {i}: {cc.timings_}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    engine.TIMERS = {}
    stats = torch.zeros(128, dtype=torch.int64, device=dev)
    t0 = time.perf_counter()
    # each fit's counters are summed after the timed region: a torch add here would put the lazy
    # load of its kernel (~70 ms, once per process) inside the second step
    step_ends, fit_totals, step_stats = [], [], []
    for i in range(args.steps):
        cc.fit(Xd)  # synchronous: returns after its host post-processing
        step_ends.append(time.perf_counter())
        fit_totals.append(cc.timings_["total"])
        step_stats.append(cc.kmeans_stats_)
        if rank == 0:
            print(f"[bench] step {i} queued", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    for st_i in step_stats:
        stats += st_i
    timers = engine.timer_summary(engine.TIMERS)
    engine.TIMERS = None

    # max over ranks (wall) and sums over ranks (work, kernel time)
    vec = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    st = stats.to(torch.float64)
    km_kernel = "cc_kmeans_batched" if cfg["d"] <= 128 else "cc_kmeans_wide"
    km_launch, km_ms = timers.get(km_kernel, (0, 0.0))
    co_launch, co_ms_launches = timers.get("cc_coassoc", (0, 0.0))
    # the per-K launches overlap on side streams (engine.coassoc_all): the band's span on the
    # fit's stream is the co-association time; the sum of launch durations is reported beside it
    co_ms = timers["coassoc_band"][1] if "coassoc_band" in timers else co_ms_launches
    ktime = torch.tensor([km_ms, float(km_launch), co_ms, co_ms_launches], dtype=torch.float64, device=dev)
    if world > 1:
        tdist.all_reduce(vec, op=tdist.ReduceOp.MAX)
        tdist.all_reduce(st, op=tdist.ReduceOp.SUM)
        tdist.all_reduce(ktime, op=tdist.ReduceOp.SUM)
    elapsed = float(vec[0])
    d = cfg["d"]
    # FLOP_KM: 2 d per distance product of Lloyd sweeps and k-means++ candidate
    # passes, counted by the kernel (st[0], st[1]); the M-step's d per (row, running problem)
    # update (st[2]) is reported separately
    flops = 2.0 * d * (float(st[0]) + float(st[1]))
    mstep_flops = d * float(st[2])
    km_ms_tot, km_launches = float(ktime[0]), max(float(ktime[1]), 1.0)
    achieved = flops / (km_ms_tot * 1e-3) / 1e12 if km_ms_tot > 0 else 0.0
    achieved_m = (flops + mstep_flops) / (km_ms_tot * 1e-3) / 1e12 if km_ms_tot > 0 else 0.0
    exec_flops = 2.0 * d * 32 * 32 * float(st[5]) if km_kernel == "cc_kmeans_batched" else 0.0
    clusterings = cfg["H"] * len(cfg["Ks"]) * args.steps
    value = clusterings / elapsed
    # co-association: OPS_M = sum_K 2 P H K per fit (channel padding and the
    # diagonal tiles' lower halves not credited) over the HIP-event time of its launches.  A
    # rehearsal (or a rank of an N-GPU run) is credited only the pairs of its own tile band.
    n_ = cfg["n"]
    if args.rehearse or world > 1:
        r_, w_ = ((int(v) for v in args.rehearse.split("/")) if args.rehearse else (rank, world))
        nt_ = (((n_ + 255) // 256) * ((n_ + 255) // 256 + 1)) // 2
        tb_, te_ = dist_shard(nt_, r_, w_)  # the fit's own tile split (api.py, dist.shard)
        P = float(band_pairs(n_, tb_, te_))
    else:
        P = n_ * (n_ - 1) / 2
    # K = 2 runs the i8 MFMA, K >= 3 the FP4 form (4x the bf16 rate): the time the credited ops
    # would take at the peak of the instruction each K actually issues
    co_ops_t = torch.tensor([sum(2.0 * P * cfg["H"] * K for K in cfg["Ks"]) * args.steps,
                             sum(2.0 * P * cfg["H"] * K / (I8_MFMA_PEAK_TOPS if K <= 2 else FP4_MFMA_PEAK_TOPS)
                                 for K in cfg["Ks"]) * args.steps],
                            dtype=torch.float64, device=dev)
    if world > 1:
        tdist.all_reduce(co_ops_t, op=tdist.ReduceOp.SUM)
    co_ops = float(co_ops_t[0])
    co_ms_tot = float(ktime[2])
    co_achieved = co_ops / (co_ms_tot * 1e-3) / 1e12 if co_ms_tot > 0 else 0.0
    co_frac_issued = float(co_ops_t[1]) / 1e12 / (co_ms_tot * 1e-3) if co_ms_tot > 0 else 0.0
    # per-config traffic files hold full single-GPU fits: not valid for a partial (rehearsal) run
    full_fit = not args.rehearse

    if rank == 0:
        traffic = load_traffic(args.config, km_kernel) if full_fit and world == 1 else None
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "resample-clusterings/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f16x3 hi/lo, f32 accumulate (k-means MFMA) / i8 (co-association MFMA)",
            "data": data,
            "config": {"workload": (f"{args.config}: {cfg.get('data', 'blobs')} n={cfg['n']} d={d} k_true={cfg['k_true']}, "
                                    f"K={cfg['Ks'][0]}..{cfg['Ks'][-1]}, H={cfg['H']}, "
                                    f"subsampling={cfg['frac']}, n_init=3, full consensus fit"),
                       "n": cfg["n"], "d": d, "K_range": [cfg["Ks"][0], cfg["Ks"][-1]],
                       "H": cfg["H"], "parallelism": f"resamples+triangle sharded over {world} GPU(s)"},
            "roofline": {
                "kernel": km_kernel,
                "bound": "mfma",
                "achieved": achieved,
                "peak": KMEANS_PEAK_TF,
                "unit": "TFLOP/s",
                "frac": checked_frac(achieved, KMEANS_PEAK_TF, "k-means"),
                "peak_note": "f16 dense MFMA peak 2516.6 TF / 3 (f32-class product = 3 f16 MFMAs)",
                "flops_note": "FLOP_KM of SURVEY.md §8d: 2*d per Lloyd and k-means++ distance product",
                "sweeps": float(st[4]), "slot_tile_row_tiles": float(st[5]),
                # executed distance products: every 32-row x 32-slot tile a sweep computes, padding
                # slots (K rounded up to 4 per problem, tiles to 32 slots) included; batched engine only
                "executed_flops_per_launch": (exec_flops / km_launches) if exec_flops else None,
                "frac_executed": (checked_frac(exec_flops / (km_ms_tot * 1e-3) / 1e12, KMEANS_PEAK_TF,
                                               "k-means executed") if exec_flops and km_ms_tot > 0 else None),
                "relocations": float(st[3]),
                "traffic": traffic,
                "flops_per_launch": flops / km_launches,
                "mstep_flops_per_launch": mstep_flops / km_launches,
                "frac_incl_mstep": checked_frac(achieved_m, KMEANS_PEAK_TF, "k-means incl. M-step"),
                "avg_launch_ms": km_ms_tot / km_launches,
            },
            "roofline_coassoc": {
                "kernel": "cc_coassoc",
                "bound": "mfma",
                "achieved": co_achieved,
                "peak": I8_MFMA_PEAK_TOPS,
                "unit": "TOP/s",
                "frac": checked_frac(co_achieved, I8_MFMA_PEAK_TOPS, "co-association"),
                "ops_per_fit": co_ops / args.steps,
                "ms_per_fit": co_ms_tot / args.steps,
                "launch_ms_sum_per_fit": float(ktime[3]) / args.steps,
                "frac_of_issued_instruction_peak": co_frac_issued,
                "issued_peak_note": "K = 2: i8 MFMA 5033 TOP/s; K >= 3: FP4 v_mfma_scale_f32_32x32x64_f8f6f4 10066 TOP/s",
                "traffic": (load_traffic(args.config, "cc_coassoc", key="bytes_per_fit")
                            if full_fit and world == 1 else None),
                "note": "the 20-bin histogram (K5) is fused into this kernel's epilogue: no HBM pass",
            },
            "kernels_ms_per_step": {k: v[1] / args.steps for k, v in timers.items()},
            "kernel_launches_per_step": {k: v[0] / args.steps for k, v in timers.items()},
            "fit_timings_s": {k: round(v, 4) for k, v in cc.timings_.items()},
            "step_ms": [round(1e3 * (b - a), 1) for a, b in zip([t0] + step_ends[:-1], step_ends)],
            "fit_total_ms": [round(1e3 * v, 1) for v in fit_totals],
            "partial": bool(cc.partial_),
        }
        if world == 1 and not args.no_consensus_roofline and not args.rehearse:
            # M, I and C at the config's n, capped at 50 000 (30 GB; C5's n would need 480 GB)
            out["roofline_consensus"] = consensus_roofline(dev, min(cfg["n"], 50_000), cfg["H"])
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg, X)
        print(json.dumps(out), flush=True)
    if world > 1:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
