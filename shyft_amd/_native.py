"""ctypes binding of the C ABI in include/shyft_hip.h (libshyft_hip.so).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded, importing this module's `lib()` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_LIB = None
_LOCK = threading.Lock()
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SHYFT_HIP_LIB") or os.path.join(_HERE, "lib", "libshyft_hip.so")

_dp = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_h = C.c_void_p

# name -> (restype, argtypes); must match include/shyft_hip.h
SIGNATURES = {
    "shyft_hip_last_error": (C.c_char_p, [_h]),
    "shyft_hip_region_create": (C.c_int, [C.c_int, C.c_size_t, C.c_int, C.POINTER(C.c_void_p)]),
    "shyft_hip_region_destroy": (None, [_h]),
    "shyft_hip_region_create_sharded": (C.c_int, [C.c_int, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "shyft_hip_region_shards": (C.c_size_t, [_h, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]),
    "shyft_hip_region_create_sharded_ex": (C.c_int, [C.c_int, C.c_size_t, C.c_void_p, C.c_size_t, C.c_uint,
                                                     C.POINTER(C.c_void_p)]),
    "shyft_hip_region_combine_path": (C.c_int, [_h]),
    "shyft_hip_region_combine_report": (C.c_char_p, [_h]),
    "shyft_hip_region_size": (C.c_size_t, [_h]),
    "shyft_hip_set_geo": (C.c_int, [_h, C.c_void_p, C.c_void_p, C.c_void_p]),
    "shyft_hip_set_parameters": (C.c_int, [_h, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p]),
    "shyft_hip_set_time_axis": (C.c_int, [_h, C.c_int64, C.c_int64, C.c_size_t, C.c_size_t]),
    "shyft_hip_set_window": (C.c_int, [_h, C.c_size_t]),
    "shyft_hip_move_window": (C.c_int, [_h, C.c_size_t, C.c_int]),
    "shyft_hip_set_collection": (C.c_int, [_h, C.c_int, C.c_int]),
    "shyft_hip_set_catchment_filter": (C.c_int, [_h, C.c_void_p, C.c_size_t]),
    "shyft_hip_set_state": (C.c_int, [_h, C.c_void_p, C.c_size_t]),
    "shyft_hip_get_state": (C.c_int, [_h, C.c_void_p, C.c_size_t]),
    "shyft_hip_copy_state": (C.c_int, [_h, _h]),
    "shyft_hip_set_forcing": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_get_forcing": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_synthetic_forcing": (C.c_int, [_h, C.c_uint64, C.c_uint64, C.c_size_t, C.c_size_t]),
    "shyft_hip_interpolate": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                        C.c_void_p]),
    "shyft_hip_interpolation_path": (C.c_int, [_h, C.c_int]),
    "shyft_hip_interpolate_btk": (C.c_int, [_h, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                            C.c_void_p, C.c_void_p]),
    "shyft_hip_btk": (C.c_int, [C.c_int, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                C.c_size_t, C.c_void_p, C.c_void_p]),
    "shyft_hip_synthetic_elevation": (C.c_int, [C.c_uint64, C.c_uint64, C.c_size_t, C.c_void_p]),
    "shyft_hip_run_cells": (C.c_int, [_h, C.c_size_t, C.c_int, C.c_int]),
    "shyft_hip_run_cells_async": (C.c_int, [_h, C.c_int, C.c_int]),
    "shyft_hip_synchronize": (C.c_int, [_h]),
    "shyft_hip_last_run_ms": (C.c_double, [_h]),
    "shyft_hip_last_interpolate_ms": (C.c_double, [_h]),
    "shyft_hip_last_run_kernel_ms": (C.c_int, [_h, C.c_void_p, C.c_int]),
    "shyft_hip_shard_run_ms": (C.c_size_t, [_h, C.c_void_p, C.c_size_t]),
    "shyft_hip_prefetch_synthetic_forcing": (C.c_int, [_h, C.c_uint64, C.c_uint64, C.c_size_t, C.c_int]),
    "shyft_hip_swap_forcing_window": (C.c_int, [_h, C.c_size_t]),
    "shyft_hip_get_series": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_get_state_series": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_statistics": (C.c_int, [_h, C.c_int, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_size_t, C.c_size_t,
                                       C.c_void_p]),
    "shyft_hip_catchment_sums": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_catchment_area_sums": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_number_of_catchments": (C.c_size_t, [_h]),
    "shyft_hip_catchment_ids": (C.c_int, [_h, C.c_void_p]),
    "shyft_hip_region_clone": (C.c_int, [_h, C.POINTER(C.c_void_p)]),
    "shyft_hip_cell_series": (C.c_int, [_h, C.c_int, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_sample_cells": (C.c_int, [_h, C.c_int, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p]),
    "shyft_hip_set_test_knob": (C.c_int, [_h, C.c_int, C.c_int64]),
    "shyft_hip_forcing_ok": (C.c_int, [_h, C.POINTER(C.c_int)]),
    "shyft_hip_set_routing_groups": (C.c_int, [_h, C.c_void_p, C.c_size_t]),
    "shyft_hip_routing_group_sums": (C.c_int, [_h, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_route": (C.c_int, [C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_int]),
    "shyft_hip_ensemble_run": (C.c_int, [_h, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int]),
    "shyft_hip_ensemble_sums": (C.c_int, [_h, C.c_int, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p, C.c_int]),
    "shyft_hip_ensemble_last_ms": (C.c_double, [_h]),
    "shyft_hip_math_selftest": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
}


def header_symbols(header: str | None = None) -> list[str]:
    """Function names declared in include/shyft_hip.h (used by the ABI test)."""
    import re
    header = header or os.path.join(os.path.dirname(_HERE), "include", "shyft_hip.h")
    src = open(header).read()
    return sorted(set(re.findall(r"\b(shyft_hip_[a-z_0-9]+)\s*\(", src)))


def lib_sha(path: str | None = None) -> str:
    """sha256 of the C ABI library file (the build identity the committed PMC summaries are keyed on:
    a summary measured on another build of the kernels is not this build's traffic)."""
    import hashlib
    h = hashlib.sha256()
    with open(path or LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def _preload_hip_runtime() -> None:
    """Load the HIP runtime PyTorch ships (if PyTorch is installed) before libshyft_hip.so.

    A process must hold ONE HIP runtime. libshyft_hip.so links libamdhip64 by soname; if it is loaded
    first, /opt/rocm's copy is mapped and a later torch.cuda initialisation (torch carries its own copy)
    finds no GPU. Mapping torch's copy first (RTLD_GLOBAL) makes both resolve to it. The torch package
    itself is not imported."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            C.CDLL(p, mode=C.RTLD_GLOBAL)
            return


def lib() -> C.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"shyft_amd: HIP library not built ({LIB_PATH}); run __graft_entry__.build()")
            _preload_hip_runtime()
            L = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _LIB = L
    return _LIB


class ShyftHipError(RuntimeError):
    """Raised for a non-zero C ABI status (maps the reference's std::runtime_error)."""


def check(status: int, handle=None) -> None:
    if status != 0:
        msg = lib().shyft_hip_last_error(handle)
        raise ShyftHipError(msg.decode() if msg else "shyft_hip error")
