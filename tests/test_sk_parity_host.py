"""The engine-precision emulation of tests/sk_parity.py (sklearn's KMeans with its Lloyd
distances at the fast engine's operand precision) reproduces sklearn's own float32 labels on
well-posed problems, so that a disagreement it shows elsewhere is a rounding sensitivity, not an
artefact of the restatement."""
import numpy as np

from tests.conftest import load_fixture
from tests.sk_parity import kmeans_at_engine_precision


def test_engine_precision_emulation_reproduces_sklearn_when_well_posed():
    from threadpoolctl import threadpool_limits

    pf = load_fixture("parity_blobs_n3000_f32")
    X, idx = pf["X"], pf["indices"]
    with threadpool_limits(1):
        for j, K in enumerate(int(k) for k in pf["K_range"]):
            if K > pf["meta"]["k_true"]:
                continue
            for h in (0, 17):
                for s in (4, 7):
                    got = kmeans_at_engine_precision(X[idx[h]], K, pf["meta"]["random_state"], 3, s=s)
                    np.testing.assert_array_equal(got, pf["labels"][j, h], err_msg=f"K={K} h={h} s={s}")
