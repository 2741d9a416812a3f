"""eray_amd — MI355X (gfx950) implementation of eray's per-pixel ray-tracing hot path.

The product is the HIP library eray_amd/lib/liberay_hip.so behind the C-ABI in
include/eray_hip.h; this package holds its sources (csrc/), its build recipe (build.py), the
ctypes binding (capi.py) and Python host tooling (objfile.py, meshgen.py, frame.py).
"""
__version__ = "0.1.0"
