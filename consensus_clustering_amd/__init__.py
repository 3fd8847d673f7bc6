"""MI355X-native consensus clustering (drop-in for trioxane/consensus_clustering's
``ConsensusClustering``): batched k-means, int8-MFMA co-association and a fused
consensus histogram on gfx950, behind the libccmi C ABI (include/ccmi.h)."""
__version__ = "0.1.0"

from .post import best_k, cdf_area, cdf_from_counts, delta_k  # noqa: F401


def __getattr__(name):
    if name == "ConsensusClustering":
        from .api import ConsensusClustering
        return ConsensusClustering
    raise AttributeError(name)
