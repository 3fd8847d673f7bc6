"""Resampling time at a config's shape: the device forms (HIP events; method swap =
cc_resample_device when n <= 65536, wide = cc_resample_device_wide) against the host replay
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
methods = ["wide"] + (["swap"] if n <= engine.resample_device_max_n() else [])
dv, hv = {k: [] for k in methods}, []
for r in range(reps + 1):
    outs = {}
    for meth in methods:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        outs[meth] = engine.resample_indices_device(0, n, m, 0, H, dev, method=meth)
        b.record()
        torch.cuda.synchronize()
        if r:
            dv[meth].append(a.elapsed_time(b))
    t0 = time.perf_counter()
    h = torch.from_numpy(engine.resample_indices(0, n, m, 0, H)).to(dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if r:
        hv.append((t1 - t0) * 1e3)
    for meth in methods:
        assert torch.equal(outs[meth], h), meth
print(f"n={n} m={m} H={H}: " + ", ".join(f"device {k} {np.round(v, 2).tolist()} ms" for k, v in dv.items())
      + f", host replay + upload {np.round(hv, 2).tolist()} ms (host threads {os.cpu_count()})", flush=True)
