"""How far sklearn's float32 KMeans is from ITSELF on the n = 3000 parity fixture.

Refits every (K, h) of tests/golden/parity_blobs_n3000_f32.npz with the reference's call
(KMeans(n_clusters=K, random_state=0, n_init=3).fit_predict(X[idx]), 1 BLAS thread), the rows
copied into a buffer at a chosen byte offset from a 64-B boundary (the only difference from the
recorded run), and reports per K: problems whose labels differ from the recording, |dPAC| and
max |dC| against the reference's own result.  This is the scale the GPU engine's float32 parity
bound (tests/test_gpu_parity_blobs.py) is set against.

    python tools/sklearn_self_parity.py OFFSET_BYTES [OFFSET_BYTES ...]
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def aligned_copy(a, offset):
    raw = np.empty(a.nbytes + 128, dtype=np.uint8)
    base = (-raw.ctypes.data) % 64 + offset
    out = raw[base:base + a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


def run(offset):
    from threadpoolctl import threadpool_limits

    from oracle import cc_oracle as O
    from tests.conftest import load_fixture

    pf = load_fixture("parity_blobs_n3000_f32")
    X, idx = pf["X"], pf["indices"]
    n, H = X.shape[0], idx.shape[0]
    I = O.cosample_matrix(idx, n)
    rows = []
    with threadpool_limits(1):
        for j, K in enumerate(int(k) for k in pf["K_range"]):
            labs = np.empty(idx.shape, dtype=np.int64)
            for h in range(H):
                labs[h] = O.kmeans_labels(aligned_copy(X[idx[h]], offset), K, 0, n_init=3)
            diff = int((labs != pf["labels"][j]).any(axis=1).sum())
            M = O.coassoc_matrix(idx, labs, K, n)
            res = O.analyse(M, I, dtype=np.uint8)
            Mr = O.coassoc_matrix(idx, pf["labels"][j].astype(np.int64), K, n)
            Cr = O.analyse(Mr, I, dtype=np.uint8)["cij"]
            rows.append((K, diff, abs(float(res["pac_area"] - pf["pac_area"][j])),
                         float(np.abs(res["cij"] - Cr).max())))
    return offset, rows


if __name__ == "__main__":
    offs = [int(a) for a in sys.argv[1:]] or [0, 4, 8, 16, 32]
    with ProcessPoolExecutor(len(offs)) as ex:
        for off, rows in ex.map(run, offs):
            print(f"offset {off:2d} B: " + "  ".join(
                f"K{K}: {d} differ, dPAC {dp:.2e}, dC {dc:.3f}" for K, d, dp, dc in rows), flush=True)
