import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith(("predict_", "parity_")))
# end-to-end parity fixtures at n = 3000 (tests/golden/make_parity_blobs.py): digests instead of
# the n x n matrices, checked by tests/test_parity_fixtures.py and tests/test_gpu_parity_blobs.py
PARITY_FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "parity_*.npz")))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (ROCm GPU) and libccmi.so")


def load_fixture(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


@pytest.fixture(params=FIXTURES)
def fixture(request):
    return load_fixture(request.param)


def digest(a) -> str:
    """SHA-256 of an array's bytes, dtype and shape (tests/golden/make_parity_blobs.py)."""
    import hashlib

    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.view(np.uint8).tobytes() + str(a.dtype).encode() + str(a.shape).encode()).hexdigest()
