"""The C-ABI library loads, exports every entry point of include/ccmi.h, and its host-native
helpers replay numpy's RandomState streams bit-exactly (no GPU needed)."""
import os
import re

import numpy as np
import pytest

from consensus_clustering_amd import _lib, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            src = open(os.path.join(ROOT, "include", fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(cc_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_symbols()
    assert len(names) >= 10
    missing = [s for s in names if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == names


def test_version_and_error():
    lib = _lib.load()
    assert b"gfx950" in lib.cc_version()
    with pytest.raises(_lib.CCMIError):
        _lib.call("cc_resample_indices", 0, 0, 1, -5, 3, None, 1)


@pytest.mark.parametrize("n,frac,seed,H", [(29, 0.8, 23, 7), (1000, 0.8, 0, 5), (4097, 0.7, 11, 3),
                                           (10, 1.0, 2**32 - 5, 4)])
def test_native_resample_matches_numpy(n, frac, seed, H):
    m = int(frac * n)
    got = engine.resample_indices(seed, n, m, 0, H)
    for h in range(H):
        ref = np.random.RandomState(seed + h).choice(n, size=m, replace=False)
        np.testing.assert_array_equal(got[h], ref)


def test_native_resample_offset_range():
    a = engine.resample_indices(5, 300, 240, 0, 6)
    b = engine.resample_indices(5, 300, 240, 2, 5, n_threads=2)
    np.testing.assert_array_equal(a[2:5], b)


def test_none_seed_raises_typeerror():
    with pytest.raises(TypeError):
        engine.resample_indices(None, 10, 8, 0, 2)


def test_native_random_sample():
    for seed in (0, 23, 4294967295):
        np.testing.assert_array_equal(engine.random_sample(seed, 1000),
                                      np.random.RandomState(seed).random_sample(1000))


def test_num_tiles():
    assert engine.num_tiles(1) == 1
    assert engine.num_tiles(256) == 1
    assert engine.num_tiles(257) == 3
    assert engine.num_tiles(50000) == 196 * 197 // 2
