"""ctypes binding of libccmi.so (the C ABI declared in include/ccmi.h).

The library is built in-tree (``make -C consensus_clustering_amd/csrc``, or
``__graft_entry__.build()``) and loaded from this package directory.  There is
no fallback: if the library is missing or fails to load, every GPU entry point
raises, so a run can never silently measure or validate a CPU path.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CCMI_LIB", os.path.join(_HERE, "libccmi.so"))

_c_int, _c_i64, _c_u32, _c_sz, _c_dbl = (ctypes.c_int, ctypes.c_int64, ctypes.c_uint32,
                                         ctypes.c_size_t, ctypes.c_double)
_vp = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/ccmi.h
SIGNATURES = {
    "cc_version": (ctypes.c_char_p, []),
    "cc_last_error": (ctypes.c_char_p, []),
    "cc_resample_indices": (_c_int, [_c_u32, _c_int, _c_int, _c_int, _c_int, _vp, _c_int]),
    "cc_resample_device_max_n": (_c_int, []),
    "cc_resample_device": (_c_int, [_c_u32, _c_int, _c_int, _c_int, _c_int, _vp, _vp]),
    "cc_resample_device_wide": (_c_int, [_c_u32, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_sz, _vp]),
    "cc_resample_device_wide_workspace_bytes": (_c_sz, [_c_int, _c_int]),
    "cc_random_sample": (_c_int, [_c_u32, _c_i64, _vp]),
    "cc_num_tiles": (_c_i64, [_c_int]),
    "cc_scatter_labels": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _vp]),
    "cc_copy_label_columns": (_c_int, [_vp, _c_i64, _c_int, _vp, _c_i64, _c_int, _c_i64, _c_int, _vp]),
    "cc_cosample": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _vp, _vp, _vp]),
    "cc_coassoc": (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_i64, _c_i64, _vp, _vp, _vp,
                            _vp, _vp, _c_int, _vp]),
    "cc_bin_table": (_c_int, [_c_int, _vp, _vp, _c_sz, _vp]),
    "cc_bin_table_bytes": (_c_sz, [_c_int]),
    "cc_bin_table_max_rows": (_c_int, []),
    "cc_bin_table_form_rows": (_c_int, [_c_int]),
    "cc_consensus": (_c_int, [_vp, _vp, _c_int, _vp, _vp]),
    "cc_kmeans_plan": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _c_int]),
    "cc_kmeans_workspace_bytes": (_c_sz, [_c_int, _c_int, _vp, _c_int, _c_int, _c_int]),
    "cc_split_f16": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "cc_kmeans_batched": (_c_int, [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int,
                                   _c_int, _c_int, _c_int, _vp, _vp, _c_int, _c_int, _c_int,
                                   _c_dbl, _vp, _c_int, _vp, _vp, _c_int, _vp, _vp, _vp, _vp,
                                   _c_sz, _c_int, _c_int, _vp]),
    "cc_kmeans_wide_workspace_bytes": (_c_sz, [_c_int, _c_int, _vp, _c_int, _c_int, _c_int]),
    "cc_kmeans_wide": (_c_int, [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int,
                                _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_dbl, _vp, _c_int,
                                _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _c_sz, _c_int, _vp]),
    "cc_build_id": (ctypes.c_char_p, []),
    "cc_bin_selftest": (_c_int, [_c_int, _vp, _vp, _vp, _vp]),
    "cc_manhattan": (_c_int, [_vp, _c_int, _c_int, _vp, _vp]),
    "cc_linkage_workspace_bytes": (ctypes.c_size_t, [_c_int]),
    "cc_linkage_nnchain": (_c_int, [_vp, _c_int, _c_int, _vp, _vp, ctypes.c_size_t, _vp]),
    "cc_linkage_mst_workspace_bytes": (ctypes.c_size_t, [_c_int]),
    "cc_linkage_mst": (_c_int, [_vp, _c_int, _vp, _vp, ctypes.c_size_t, _vp]),
    "cc_linkage_check": (_c_int, [_vp, ctypes.c_size_t, _vp]),
    "cc_kmeans_f64_workspace_bytes": (_c_sz, [_c_int, _c_int, _vp, _c_int, _c_int, _c_int]),
    "cc_kmeans_f64": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp,
                               _c_int, _c_int, _c_int, _c_dbl, _vp, _c_int, _vp, _vp, _c_int, _vp,
                               _vp, _vp, _c_sz, _c_int, _vp]),
    "cc_kpp_tables": (_c_int, [_vp, _c_int, _c_int, _c_u32, _c_int, _c_int, _vp, _c_int, _vp]),
    "cc_prepare_rows_scratch_bytes": (_c_sz, [_c_int, _c_int]),
    "cc_prepare_rows": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "cc_kmeans_fit_workspace_bytes": (_c_sz, [_c_int, _c_int, _c_int, _c_int, _vp, _c_int, _c_int,
                                              _c_int]),
    "cc_kmeans_fit": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int,
                               _c_int, _c_int, _c_dbl, _c_u32, _c_int, _vp, _c_int, _vp, _vp, _vp,
                               _c_sz, _vp]),
}

_CSRC = os.path.join(_HERE, "csrc")
_INCLUDE = os.path.join(os.path.dirname(_HERE), "include", "ccmi.h")


def source_build_id() -> str:
    """The build id the csrc Makefile embeds: SHA-256 prefix over the sources in its order."""
    names = sorted(f for f in os.listdir(_CSRC) if f.endswith((".hip", ".cpp", ".h", ".hpp")))
    h = hashlib.sha256()
    for path in [os.path.join(_CSRC, f) for f in names] + [_INCLUDE, os.path.join(_CSRC, "Makefile")]:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]

_lock = threading.Lock()
_lib = None


class CCMIError(RuntimeError):
    """A libccmi entry point returned a non-zero status."""


def load():
    """Load libccmi.so once; raise loudly if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise CCMIError(
                f"libccmi.so not found at {LIB_PATH}: build it with "
                "`make -C consensus_clustering_amd/csrc` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if "CCMI_LIB" in os.environ and not hasattr(lib, name):
                continue  # an explicitly named (older / diagnostic) build for A/B timing
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        # provenance: the library must be built from exactly the sources next to it, with the
        # default flags (no diagnostic -D variant), unless CCMI_LIB names one explicitly
        if "CCMI_LIB" not in os.environ and os.path.isdir(_CSRC):
            built = lib.cc_build_id().decode()
            want = source_build_id()
            if built != want:
                raise CCMIError(
                    f"stale libccmi.so (built from {built}, sources are {want}): rebuild with "
                    "`make -C consensus_clustering_amd/csrc` or __graft_entry__.build()")
            if b"-D" in lib.cc_version():
                raise CCMIError("libccmi.so is a diagnostic build (-D flags): rebuild it")
        _lib = lib
        return lib


def check(rc: int, fn: str):
    if rc != 0:
        msg = load().cc_last_error().decode(errors="replace")
        raise CCMIError(f"{fn} failed ({rc}): {msg}")


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    check(rc, name)
    return rc


def ptr(t) -> int:
    """Raw device/host pointer of a torch tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data
