"""Worker side of the hybrid path's parallel host fits (api.host_fit_predict, CC.py:185-195).

Kept free of torch and of the GPU modules: a joblib process worker unpickles the task function
by importing its module, and importing the engine would import torch (seconds per worker, a
minute on a freshly paged-in image) before the first fit."""
import numpy as np


def fit_predict_one(clusterer, Xs):
    """``clusterer.fit_predict(Xs)`` as CC.py:282 calls it, labels as an array."""
    return np.asarray(clusterer.fit_predict(Xs))


def fit_predict_chunk(clusterer, Xs_list):
    """The labels of several resamples, one fit after the other on the task's own clusterer."""
    return [fit_predict_one(clusterer, Xs) for Xs in Xs_list]
