"""Phase cycles of the co-association kernel (diagnostic -DCC_CO_STAMPS build).

    CCMI_LIB=consensus_clustering_amd/libccmi_costamps.so python tools/co_stamps.py [config] [K ...]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from consensus_clustering_amd import _lib, engine, post  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
Ks = [int(k) for k in sys.argv[2:]] or cfg["Ks"]
n, H = cfg["n"], cfg["H"]
dev = torch.device("cuda")
Hpad = engine.pad_h(H)
g = torch.Generator(device=dev).manual_seed(0)
labels = engine.new_label_matrix(1, n, Hpad, dev)
samp = torch.rand((n, H), generator=g, device=dev) < cfg["frac"]
lib = _lib.load()
fn = lib.cc_co_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
nt = engine.num_tiles(n)
edges = engine.edges_device(dev)
counts = torch.zeros((post.N_BINS,), dtype=torch.int64, device=dev)
names = ["prologue", "main", "epi_setup", "binning", "reduce"]
for K in Ks:
    lab = torch.randint(0, K, (n, H), generator=g, device=dev, dtype=torch.int32).to(torch.uint8)
    labels[0, :, :H] = torch.where(samp, lab, torch.full_like(lab, 255))
    I_tiles, _ = engine.cosample(labels[0], n, Hpad, 0, nt, want_full=False)
    engine.coassoc(labels[0], n, Hpad, K, 0, nt, I_tiles, edges, counts)
    torch.cuda.synchronize()
    fn(buf, 1)
    engine.coassoc(labels[0], n, Hpad, K, 0, nt, I_tiles, edges, counts)
    torch.cuda.synchronize()
    fn(buf, 1)
    tot = sum(buf[:5])
    print(f"K={K}: per tile " + " ".join(f"{nm} {buf[i] / nt / 1e3:.1f}k" for i, nm in enumerate(names))
          + f" | total {tot / nt / 1e3:.1f}k cycles", flush=True)
