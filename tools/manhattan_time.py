"""cc_manhattan alone (HIP events) on a random float32 C [n, n], for build variants (CCMI_LIB).

    python tools/manhattan_time.py [n] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hashlib  # noqa: E402

import torch  # noqa: E402

from consensus_clustering_amd import engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = engine.require_gpu()
C = torch.rand((n, n), generator=torch.Generator(device=dev).manual_seed(0), device=dev)
ts = []
for r in range(reps + 1):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    D = engine.manhattan(C)
    b.record()
    torch.cuda.synchronize()
    if r:
        ts.append(round(a.elapsed_time(b), 1))
    dig = hashlib.sha256(D[:: max(1, n // 512)].cpu().numpy().tobytes()).hexdigest()[:16]
    del D
print(os.path.basename(os.environ.get("CCMI_LIB", "libccmi.so")), f"manhattan n={n} ms", ts, "digest", dig, flush=True)
