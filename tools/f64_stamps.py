"""Diagnostic: thread 0's wall-clock split of the float64 k-means phases (stamps build,
libccmi_f64stamps.so, -DCC_F64_STAMPS), per config shape and resample count.

    python tools/f64_stamps.py CONFIG H [CONFIG H ...]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CCMI_LIB", os.path.join(ROOT, "consensus_clustering_amd", "libccmi_f64stamps.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS, SEED, make_blobs_f32  # noqa: E402
from consensus_clustering_amd import _lib, engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans  # noqa: E402

NAMES = ["setup", "k-means++", "E-step", "counts+lists", "M-sums", "reloc+avg+shift", "final+inertia",
         "unit fetch/idle"]
dev = engine.require_gpu()
lib = _lib.load()
fn = lib.cc_kmeans_f64_stamps
fn.argtypes = [ctypes.c_void_p]
args = sys.argv[1:]
for i in range(0, len(args), 2):
    name, H = args[i], int(args[i + 1])
    cfg = CONFIGS[name]
    X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"], seed=SEED).astype(np.float64)
    X += np.random.default_rng(0).normal(scale=0.05, size=X.shape)
    n, d = X.shape
    m = int(cfg["frac"] * n)
    idx_d = torch.from_numpy(engine.resample_indices(SEED, n, m, 0, H)).to(dev)
    X64 = torch.from_numpy(X).to(dev)
    L = engine.new_label_matrix(len(cfg["Ks"]), n, engine.pad_h(H), dev)
    bk = BatchedKMeans(cfg["Ks"], n_init=3, random_state=SEED)
    out = np.zeros(16, dtype=np.uint64)
    fn(out.ctypes.data)  # zero
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    bk.run_f64(X64, idx_d, n, H, m, 0, H, L)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    fn(out.ctypes.data)
    tot = float(out[:8].sum())
    print(f"{name} H={H} units={H * len(cfg['Ks'])} workgroups={int(out[9])}: {ms:.1f} ms; "
          f"Lloyd iterations {int(out[8])}")
    tot += float(out[10:13].sum())
    for q in list(range(8)) + [10, 11, 12]:
        name = NAMES[q] if q < 8 else ["  k-means++ search", "  k-means++ distances", "  k-means++ potentials"][q - 10]
        print(f"  {name:22s} {100 * out[q] / tot:5.1f} %   {out[q] / 100e3 / max(int(out[9]), 1):9.1f} ms per workgroup")
    # per-unit timeline of the launch (units dealt in order: kind-major, resample-minor)
    nu = H * len(cfg["Ks"])
    ut = np.zeros((nu, 3), dtype=np.uint64)
    if hasattr(lib, "cc_kmeans_f64_unit_times") and nu <= 16384:
        lib.cc_kmeans_f64_unit_times(ctypes.c_void_p(ut.ctypes.data), nu)
        used = ut[:, 1] > 0
        ut = ut[used].astype(np.float64)
        t0 = ut[:, 0].min()
        st, en = (ut[:, 0] - t0) / 100e3, (ut[:, 1] - t0) / 100e3
        dur = en - st
        wall = en.max()
        ends = np.array([en[ut[:, 2] == w].max() for w in np.unique(ut[:, 2])])
        print(f"  timeline: {int(used.sum())} units, last end {wall:.1f} ms; workgroup finish "
              f"p10/p50/p90 {np.percentile(ends, 10):.1f}/{np.percentile(ends, 50):.1f}/"
              f"{np.percentile(ends, 90):.1f} ms; busy {100 * dur.sum() / (len(ends) * wall):.1f} %")
        order = np.argsort(-dur)[:8]
        print("  longest units (index, start, duration ms): " +
              ", ".join(f"{np.flatnonzero(used)[i]}@{st[i]:.0f}+{dur[i]:.0f}" for i in order))
        late = np.argsort(-st)[:5]
        print("  last started (index, start, duration ms): " +
              ", ".join(f"{np.flatnonzero(used)[i]}@{st[i]:.0f}+{dur[i]:.0f}" for i in late))
        # mean duration per unit kind (rows of H consecutive units)
        idx_used = np.flatnonzero(used)
        kinds = idx_used // H
        print("  per kind mean/max ms: " + " ".join(
            f"{k}:{dur[kinds == k].mean():.0f}/{dur[kinds == k].max():.0f}" for k in np.unique(kinds)))
    sys.stdout.flush()
