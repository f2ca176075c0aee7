"""bitalosdb_amd -- MI355X-native bithash value-log block codec.

The product is libbithashgpu.so (HIP kernels for gfx950 behind the C-ABI in
include/bithashgpu.h).  This package holds its sources (csrc/), the ctypes
binding (_lib.py) and a host-side mirror of the reference's codec surface
(codec.py) used by tests, the smoke check and the benchmark.
"""
__all__ = ["_lib"]
