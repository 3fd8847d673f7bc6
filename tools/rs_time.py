"""Resampling time at a config's shape: cc_resample_device (HIP events) against the host replay
cc_resample_indices plus its upload (wall clock).

    python tools/rs_time.py [config] [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = engine.require_gpu()
n, H = cfg["n"], cfg["H"]
m = int(cfg["frac"] * n)
dv, hv = [], []
for r in range(reps + 1):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    d = engine.resample_indices_device(0, n, m, 0, H, dev)
    b.record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = torch.from_numpy(engine.resample_indices(0, n, m, 0, H)).to(dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if r:
        dv.append(a.elapsed_time(b))
        hv.append((t1 - t0) * 1e3)
assert torch.equal(d, h)
print(f"n={n} m={m} H={H}: device {np.round(dv, 2).tolist()} ms, host replay + upload {np.round(hv, 2).tolist()} ms "
      f"(host threads {os.cpu_count()})", flush=True)
