"""ctypes binding of libesgd.so (the C ABI in include/esgd.h and include/esgd_ff.h).

The product path has no CPU fallback: if the HIP library cannot be loaded, or a call
needs a device that is not there, this module raises.  PyTorch (when importable) is
imported *before* the library so that the process holds exactly one HIP runtime
(torch ships its own libamdhip64.so.7; the dynamic loader then binds libesgd.so to
that copy through the shared soname).
"""
from __future__ import annotations

import array
import ctypes as C
import os

try:  # one HIP runtime per process: let torch's copy be the one (see module doc)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C path
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ESGD_LIB", os.path.join(_HERE, "libesgd.so"))

SUCCESS, ERROR, INVALID_ARG, ENOMEM, NO_DEVICE = 0, -1, -2, -4, -6
INT32, INT64, DOUBLE, FLOAT, BF16 = 0, 1, 2, 3, 16
MAX_FANIN = 8


class EsgdError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"libesgd error {rc}: {msg}")
        self.rc = rc


_vp, _sz, _u64, _i, _f = C.c_void_p, C.c_size_t, C.c_uint64, C.c_int, C.c_float

# name -> (restype, argtypes)
_SIGS = {
    "esgd_last_error": (C.c_char_p, []),
    "esgd_version": (_i, []),
    "esgd_dtype_size": (_sz, [_i]),
    "esgd_device_count": (_i, [C.POINTER(_i)]),
    "esgd_set_device": (_i, [_i]),
    "esgd_get_device": (_i, [C.POINTER(_i)]),
    "esgd_device_arch": (_i, [_i, C.c_char_p, _sz]),
    "esgd_malloc": (_i, [C.POINTER(_vp), _sz]),
    "esgd_free": (_i, [_vp]),
    "esgd_memory_stats": (_i, [C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u64)]),
    "esgd_host_alloc": (_i, [C.POINTER(_vp), _sz]),
    "esgd_host_free": (_i, [_vp]),
    "esgd_host_register": (_i, [_vp, _sz]),
    "esgd_host_unregister": (_i, [_vp]),
    "esgd_memcpy_async": (_i, [_vp, _vp, _sz, _i, _vp]),
    "esgd_memset_async": (_i, [_vp, _i, _sz, _vp]),
    "esgd_stream_create": (_i, [C.POINTER(_vp)]),
    "esgd_stream_destroy": (_i, [_vp]),
    "esgd_stream_synchronize": (_i, [_vp]),
    "esgd_device_synchronize": (_i, []),
    "esgd_event_create": (_i, [C.POINTER(_vp)]),
    "esgd_event_destroy": (_i, [_vp]),
    "esgd_event_record": (_i, [_vp, _vp]),
    "esgd_event_synchronize": (_i, [_vp]),
    "esgd_event_elapsed_ms": (_i, [_vp, _vp, C.POINTER(_f)]),
    "esgd_stream_wait_event": (_i, [_vp, _vp]),
    "esgd_reduce": (_i, [_i, _i, C.POINTER(_vp), _vp, _u64, _vp]),
    "esgd_reduce_host": (_i, [_i, _i, C.POINTER(_vp), _vp, _u64, _vp]),
    "esgd_reduce_scaled": (_i, [_i, _i, C.POINTER(_vp), _vp, _u64, _f, _vp]),
    "esgd_vsum": (_i, [_i, _vp, _vp, _vp, _u64, _vp]),
    "esgd_fill_uniform_f32": (_i, [_u64, _i, _vp, _u64, _vp]),
    "esgd_pack_div": (_i, [_i, C.POINTER(_vp), C.POINTER(_u64), _vp, _f, _vp]),
    "esgd_unpack": (_i, [_i, C.POINTER(_vp), C.POINTER(_u64), _vp, _vp]),
    "esgd_fill_uniform_bf16": (_i, [_u64, _i, _vp, _u64, _vp]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libesgd.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EsgdError(ERROR, f"{LIB_PATH} not built (run `make lib` or __graft_entry__.build())")
        handle = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype, fn.argtypes = res, args
        _lib = handle
        _bind_extra(handle)
    return _lib


_EXTRA_BINDERS = []


def register_signatures(binder):
    """Sub-modules add their own prototypes (ff.h, deep500) through this hook."""
    _EXTRA_BINDERS.append(binder)
    if _lib is not None:
        binder(_lib)


def _bind_extra(handle):
    for b in _EXTRA_BINDERS:
        b(handle)


def last_error() -> str:
    msg = lib().esgd_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "") -> int:
    if rc != SUCCESS:
        raise EsgdError(rc, f"{what}: {last_error()}" if what else last_error())
    return rc


def device_count() -> int:
    n = C.c_int(0)
    check(lib().esgd_device_count(C.byref(n)), "esgd_device_count")
    return n.value


def dtype_size(dtype: int) -> int:
    return int(lib().esgd_dtype_size(dtype))


def ptr_array(ptrs):
    """A C array of pointers from Python ints, through array('Q') (about 3x cheaper than
    ctypes' element-wise conversion: the optimizer passes 161-entry groups every step).  The
    ctypes array keeps the buffer alive."""
    buf = array.array("Q", ptrs)
    if not buf:
        return (C.c_void_p * 1)()
    return (C.c_void_p * len(buf)).from_buffer(buf)
