"""esgd — MI355X-native gradient-bucket reduction for eager-SGD (host-side package).

Layers:
  _lib     ctypes binding of libesgd.so (C ABI: include/esgd.h, esgd_ff.h, esgd_deep500.h)
  device   device buffers / streams / events and the reduction launches
"""
from ._lib import (BF16, DOUBLE, FLOAT, INT32, INT64, MAX_FANIN, EsgdError,  # noqa: F401
                   check, device_count, lib)

__version__ = "0.1.0"
