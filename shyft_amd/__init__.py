"""shyft_amd — MI355X-native engine for Shyft's distributed-cell hydrology hot path
(region_model::run_interpolation / run_cells).

Layers:
  include/shyft_hip.h        C ABI (the drop-in boundary)
  shyft_amd/csrc/            HIP kernels for gfx950 + the C ABI implementation
  shyft_amd/region.py        thin Python owner of a region handle
  shyft_amd/synthetic.py     deterministic synthetic workload
"""
__version__ = "0.1.0"
