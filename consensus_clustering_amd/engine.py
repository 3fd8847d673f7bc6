"""Device engine: torch-ROCm tensors as raw buffers around the libccmi C ABI.

Torch is plumbing here (device memory, the current HIP stream, torch.distributed);
every count, label and histogram is produced by the gfx950 kernels in
``csrc/`` through ``_lib``.  No function in this module has a CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .post import N_BINS, bin_edges32

TILE = 256
HALIGN = 128  # resample padding of the sample-major label matrix (Hpad % 128 == 0)


def require_gpu(device=None) -> torch.device:
    """The torch device to run on; raises if there is no GPU or no libccmi.so."""
    if not torch.cuda.is_available():
        raise _lib.CCMIError(
            "consensus_clustering_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    _lib.load()
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


# Optional per-launch HIP-event timing (bench.py): {kernel name: [(start, end), ...]}.
TIMERS = None


class timed:
    """Record HIP events around a launch on the current stream when TIMERS is enabled."""

    def __init__(self, name):
        self.name = name
        self.ev = None

    def __enter__(self):
        if TIMERS is not None:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()
        return self

    def __exit__(self, *exc):
        if self.ev is not None:
            self.ev[1].record()
            TIMERS.setdefault(self.name, []).append(self.ev)
        return False


def timer_summary(timers) -> dict:
    """{name: (launches, total ms)} after a synchronize."""
    return {k: (len(v), sum(a.elapsed_time(b) for a, b in v)) for k, v in timers.items()}


def pad_h(H: int) -> int:
    return ((H + HALIGN - 1) // HALIGN) * HALIGN


def num_tiles(n: int) -> int:
    return int(_lib.load().cc_num_tiles(int(n)))


# ---------------------------------------------------------------- host-native RNG

def resample_indices(seed: int, n: int, m: int, h_begin: int, h_end: int, n_threads: int = 0) -> np.ndarray:
    """int32 [h_end-h_begin, m]: RandomState(seed+h).choice(n, m, replace=False) (CC.py:231-239)."""
    if seed is None:
        # the reference computes `self.random_state + i` (CC.py:232)
        raise TypeError("unsupported operand type(s) for +: 'NoneType' and 'int'")
    seed = int(seed)
    if seed < 0 or seed + h_end - 1 > 2**32 - 1:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    out = np.empty((h_end - h_begin, m), dtype=np.int32)
    _lib.call("cc_resample_indices", ctypes.c_uint32(seed), h_begin, h_end, n, m,
              out.ctypes.data, n_threads)
    return out


# workspace cap of the swap-partner resampling (resamples run in batches that fit; 4 GiB holds
# every resample of C5 in one batch, one workgroup per resample across the whole GPU)
RESAMPLE_WIDE_WS = 4 << 30


RESAMPLE_SWAP_MAX_AUTO = 16384  # 'auto' uses the LDS swap chain up to this n, the wide form above


def resample_indices_device(seed: int, n: int, m: int, h_begin: int, h_end: int, device,
                            out: torch.Tensor | None = None, method: str = "auto") -> torch.Tensor:
    """int32 [h_end-h_begin, m] on the device: the same draws as resample_indices.
    method 'swap': cc_resample_device (the shuffle simulated in LDS; n <= 65536); 'wide':
    cc_resample_device_wide (any n, resolved from the swap partners); 'auto': wide when
    n > 16384 (faster from there: C3 n = 50k 7.3 against 24.7 ms; equal at n = 10k) else swap.  `out`: a contiguous int32 device tensor of that shape to fill (e.g. a
    row slice of the full [H, m] matrix)."""
    if seed is None:
        raise TypeError("unsupported operand type(s) for +: 'NoneType' and 'int'")
    seed = int(seed)
    if seed < 0 or seed + h_end - 1 > 2**32 - 1:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    if out is None:
        out = torch.empty((h_end - h_begin, m), dtype=torch.int32, device=device)
    elif (tuple(out.shape) != (h_end - h_begin, m) or out.dtype != torch.int32 or not out.is_contiguous()
          or not out.is_cuda):
        raise ValueError("out must be a contiguous int32 device tensor of shape [h_end - h_begin, m]")
    if method == "auto":
        method = "wide" if n > RESAMPLE_SWAP_MAX_AUTO else "swap"
    if method == "swap":
        _lib.call("cc_resample_device", ctypes.c_uint32(seed), h_begin, h_end, n, m,
                  out.data_ptr() if out.numel() else None, stream_ptr(device))
    elif method == "wide":
        lib = _lib.load()
        nh = max(h_end - h_begin, 1)
        per = int(lib.cc_resample_device_wide_workspace_bytes(n, 1))
        nb = max(1, min(nh, RESAMPLE_WIDE_WS // max(per, 1)))
        ws = torch.empty(per * nb, dtype=torch.uint8, device=device)
        _lib.call("cc_resample_device_wide", ctypes.c_uint32(seed), h_begin, h_end, n, m,
                  out.data_ptr() if out.numel() else None, ws.data_ptr(), ws.numel(),
                  stream_ptr(device))
    else:
        raise ValueError("method must be 'auto', 'swap' or 'wide'")
    return out


def resample_device_max_n() -> int:
    """Largest n of the LDS shuffle (cc_resample_device); the wide form has no limit."""
    return int(_lib.load().cc_resample_device_max_n())


def random_sample(seed: int, count: int) -> np.ndarray:
    """RandomState(seed).random_sample(count) via the native MT19937."""
    out = np.empty(count, dtype=np.float64)
    _lib.call("cc_random_sample", ctypes.c_uint32(int(seed)), int(count),
              out.ctypes.data if count else None)
    return out


# ---------------------------------------------------------------- label matrices

def new_label_matrix(nK: int, n: int, Hpad: int, device) -> torch.Tensor:
    """uint8 [nK, n, Hpad] filled with 0xFF (= not sampled)."""
    return torch.full((nK, n, Hpad), 0xFF, dtype=torch.uint8, device=device)


def scatter_labels(idx_hm: torch.Tensor, labels_hm, n: int, out_nh: torch.Tensor, h_offset: int = 0):
    """out_nh[idx[h, r], h_offset + h] = labels[h, r] (or 0 when labels_hm is None)."""
    H, m = idx_hm.shape
    assert idx_hm.dtype == torch.int32 and idx_hm.is_contiguous()
    assert out_nh.dtype == torch.uint8 and out_nh.dim() == 2 and out_nh.shape[0] == n
    assert out_nh.stride(1) == 1
    ldl = out_nh.stride(0)
    if labels_hm is not None:
        assert labels_hm.dtype == torch.int32 and tuple(labels_hm.shape) == (H, m)
        labels_hm = labels_hm.contiguous()
    if H == 0:  # a rank that owns no resample (dist.shard) has nothing to place
        return
    base = out_nh[:, h_offset:]
    _lib.call("cc_scatter_labels", _lib.ptr(idx_hm), _lib.ptr(labels_hm), H, m, n,
              base.data_ptr(), ldl, stream_ptr())


def copy_label_columns(src: torch.Tensor, col_src: int, dst: torch.Tensor, col_dst: int, width: int):
    """dst[..., col_dst:col_dst+width] = src[..., col_src:col_src+width] for two device uint8
    label matrices of the same leading shape (cc_copy_label_columns, one launch)."""
    assert src.dtype == torch.uint8 and dst.dtype == torch.uint8 and src.is_cuda and dst.is_cuda
    assert src.is_contiguous() and dst.is_contiguous() and src.shape[:-1] == dst.shape[:-1]
    rows = src.numel() // src.shape[-1] if src.numel() else 0
    _lib.call("cc_copy_label_columns", src.data_ptr(), src.shape[-1], int(col_src), dst.data_ptr(),
              dst.shape[-1], int(col_dst), rows, int(width), stream_ptr(src.device))


# ---------------------------------------------------------------- co-sampling / co-association

def cosample(labels_nh: torch.Tensor, n: int, Hpad: int, tile_begin: int, tile_end: int,
             want_full: bool = False):
    """I tiles (uint16 accumulator order) for [tile_begin, tile_end), optional full int32 I."""
    dev = labels_nh.device
    ntl = tile_end - tile_begin
    I_tiles = torch.empty((max(ntl, 0), TILE * TILE), dtype=torch.int16, device=dev)
    I_full = torch.zeros((n, n), dtype=torch.int32, device=dev) if want_full else None
    with timed("cc_cosample"):
        _lib.call("cc_cosample", labels_nh.data_ptr(), n, labels_nh.stride(0), Hpad, tile_begin,
                  tile_end, I_tiles.data_ptr(), _lib.ptr(I_full), stream_ptr())
    return I_tiles, I_full


def edges_device(device) -> torch.Tensor:
    return torch.from_numpy(bin_edges32().copy()).to(device)


_BIN_TABLES = {}


def bin_table(device, rows: int):
    """Cached cc_bin_table thresholds for co-sampling counts [0, rows), or None when the table
    is too large to stage on chip (cc_coassoc then bins by division)."""
    if rows > _lib.load().cc_bin_table_max_rows():
        return None
    key = (str(device), rows)
    t = _BIN_TABLES.get(key)
    if t is None:
        nbytes = int(_lib.load().cc_bin_table_bytes(rows))
        t = torch.zeros(nbytes // 2, dtype=torch.int16, device=device)
        _lib.call("cc_bin_table", rows, edges_device(device).data_ptr(), t.data_ptr(), nbytes,
                  stream_ptr())
        _BIN_TABLES[key] = t
    return t


def coassoc(labels_nh: torch.Tensor, n: int, Hpad: int, K: int, tile_begin: int, tile_end: int,
            I_tiles: torch.Tensor, edges: torch.Tensor, counts: torch.Tensor,
            M_full: torch.Tensor = None, use_table: bool = True):
    """Accumulate the strict-upper-pair histogram of C for one K into counts (int64[20])."""
    assert counts.dtype == torch.int64 and counts.numel() == N_BINS
    tab = bin_table(labels_nh.device, Hpad + 1) if use_table else None
    with timed("cc_coassoc"):
        _lib.call("cc_coassoc", labels_nh.data_ptr(), n, labels_nh.stride(0), Hpad, int(K),
                  tile_begin, tile_end, I_tiles.data_ptr(), edges.data_ptr(), counts.data_ptr(),
                  _lib.ptr(M_full), _lib.ptr(tab), Hpad + 1 if tab is not None else 0,
                  stream_ptr())


_SIDE_STREAMS = {}


def side_streams(device, count: int):
    """`count` cached HIP streams of `device` for independent launches (the per-K co-association
    launches of a fit): a launch covers only the tiles of one K, so at small n its last round of
    tiles leaves CUs idle that the next K's launch can fill."""
    key = str(device)
    have = _SIDE_STREAMS.setdefault(key, [])
    while len(have) < count:
        have.append(torch.cuda.Stream(device=device))
    return have[:count]


def coassoc_all(labels: torch.Tensor, n: int, Hpad: int, Ks, tile_begin: int, tile_end: int,
                I_tiles: torch.Tensor, counts: torch.Tensor, M_full=None, streams: int = 2):
    """coassoc for every K (labels[k], counts[k], M_full[k]), the launches dealt round robin over
    `streams` side streams forked from and joined back into the current stream.  The K are
    independent (own label matrix, own counters), so the results do not depend on the overlap."""
    dev = labels.device
    edges = edges_device(dev)
    bin_table(dev, Hpad + 1)  # staged once on the current stream, before any side stream reads it
    main = torch.cuda.current_stream(dev)
    if streams <= 1 or len(Ks) <= 1:
        for k, K in enumerate(Ks):
            coassoc(labels[k], n, Hpad, K, tile_begin, tile_end, I_tiles, edges, counts[k],
                    None if M_full is None else M_full[k])
        return
    ss = side_streams(dev, min(int(streams), len(Ks)))
    with timed("coassoc_band"):
        for s in ss:
            s.wait_stream(main)
        for k, K in enumerate(Ks):
            with torch.cuda.stream(ss[k % len(ss)]):
                coassoc(labels[k], n, Hpad, K, tile_begin, tile_end, I_tiles, edges, counts[k],
                        None if M_full is None else M_full[k])
        for s in ss:
            main.wait_stream(s)


def consensus(M: torch.Tensor, I: torch.Tensor) -> torch.Tensor:
    n = M.shape[0]
    C = torch.empty((n, n), dtype=torch.float32, device=M.device)
    _lib.call("cc_consensus", M.data_ptr(), I.data_ptr(), n, C.data_ptr(), stream_ptr())
    return C


LINKAGE_METHODS = {"average": 0, "complete": 1, "weighted": 2}  # CC_LINK_* (include/ccmi.h)


def linkage_raw(D: torch.Tensor, method: str) -> torch.Tensor:
    """nn_chain's merges (x, y, distance, size) in merge order, on the device (D overwritten)."""
    assert D.dtype == torch.float64 and D.dim() == 2 and D.shape[0] == D.shape[1] and D.is_contiguous()
    n = D.shape[0]
    Z = torch.empty((n - 1, 4), dtype=torch.float64, device=D.device)
    lib = _lib.load()
    ws = torch.empty(int(lib.cc_linkage_workspace_bytes(n)), dtype=torch.uint8, device=D.device)
    _lib.call("cc_linkage_nnchain", D.data_ptr(), n, LINKAGE_METHODS[method], Z.data_ptr(), ws.data_ptr(),
              ws.numel(), stream_ptr())
    _lib.call("cc_linkage_check", ws.data_ptr(), ws.numel(), stream_ptr())
    return Z


def linkage(D: torch.Tensor, method: str) -> np.ndarray:
    """scipy.cluster.hierarchy.linkage of the symmetric float64 [n, n] distances D (device; D is
    overwritten) for method in LINKAGE_METHODS: scipy's nn_chain on the device
    (cc_linkage_nnchain), then linkage()'s stable sort of the merges by distance and its union-find
    relabelling (scipy/cluster/_hierarchy.pyx: nn_chain, label) on the host.  Returns Z [n-1, 4]."""
    n = D.shape[0]
    Z = linkage_raw(D, method)
    from .post import linkage_finish

    return linkage_finish(Z.cpu().numpy(), n)


def linkage_single(D: torch.Tensor) -> np.ndarray:
    """sklearn's single-linkage tree of the rows behind the symmetric float64 [n, n] distances D
    (device, read only): mst_linkage_core's Prim edges on the device (cc_linkage_mst), then the
    stable sort and _single_linkage_label on the host (post.single_linkage_finish).  Z [n-1, 4]."""
    assert D.dtype == torch.float64 and D.dim() == 2 and D.shape[0] == D.shape[1] and D.is_contiguous()
    n = D.shape[0]
    out = torch.empty((n - 1, 3), dtype=torch.float64, device=D.device)
    ws = torch.empty(int(_lib.load().cc_linkage_mst_workspace_bytes(n)), dtype=torch.uint8, device=D.device)
    _lib.call("cc_linkage_mst", D.data_ptr(), n, out.data_ptr(), ws.data_ptr(), ws.numel(), stream_ptr())
    _lib.call("cc_linkage_check", ws.data_ptr(), ws.numel(), stream_ptr())
    from .post import single_linkage_finish

    return single_linkage_finish(out.cpu().numpy(), n)


def manhattan(C: torch.Tensor) -> torch.Tensor:
    """float64 [n, n] manhattan distances between the rows of the float32 [n, n] C."""
    assert C.dtype == torch.float32 and C.dim() == 2 and C.is_contiguous()
    n, d = C.shape
    D = torch.empty((n, n), dtype=torch.float64, device=C.device)
    _lib.call("cc_manhattan", C.data_ptr(), n, d, D.data_ptr(), stream_ptr())
    return D
