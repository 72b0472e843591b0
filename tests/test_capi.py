"""The C-ABI library loads and exports every symbol include/shyft_hip.h declares
(no compute calls: CPU-only check)."""
import ctypes as C
import os

from shyft_amd import _native


def test_library_exports_every_header_symbol():
    assert os.path.exists(_native.LIB_PATH), "libshyft_hip.so not built; run __graft_entry__.build()"
    L = C.CDLL(_native.LIB_PATH)
    names = _native.header_symbols()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # every declared function has a ctypes signature in the Python binding
    assert set(names) == set(_native.SIGNATURES), set(names) ^ set(_native.SIGNATURES)


def test_errors_are_reported_without_a_handle():
    L = _native.lib()
    h = C.c_void_p()
    assert L.shyft_hip_region_create(99, 10, 0, C.byref(h)) != 0
    assert b"unsupported" in L.shyft_hip_last_error(None)


def test_synthetic_elevation_matches_numpy():
    import numpy as np
    from shyft_amd import synthetic
    z = np.empty(1000)
    L = _native.lib()
    assert L.shyft_hip_synthetic_elevation(synthetic.SEED, 12345, 1000, z.ctypes.data_as(C.c_void_p)) == 0
    assert np.array_equal(z, synthetic.elevation(1000, synthetic.SEED, 12345))
