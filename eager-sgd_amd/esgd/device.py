"""Thin Python handles over libesgd's device plumbing and the reduction kernels.

Nothing here computes on the host: every reduction is a HIP launch through the C ABI
(esgd_reduce / esgd_vsum).  Buffers are raw device allocations owned by libesgd, so
the module works without PyTorch; `as_ptr` also accepts torch tensors (data_ptr()).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib

NP_DTYPE = {
    _lib.INT32: np.int32,
    _lib.INT64: np.int64,
    _lib.DOUBLE: np.float64,
    _lib.FLOAT: np.float32,
    _lib.BF16: np.uint16,  # raw bf16 bits
}


def as_ptr(x) -> int:
    dp = getattr(x, "data_ptr", None)   # torch tensors first: the per-step group calls
    if dp is not None:
        return int(dp())
    if isinstance(x, int):
        return x
    if hasattr(x, "ptr"):
        return int(x.ptr)
    raise TypeError(f"cannot take a device pointer of {type(x)!r}")


def ptr_array_of(xs):
    """_lib.ptr_array of as_ptr(x) for every x: torch tensors' data_ptr() in one
    comprehension (161 of them in 21 us; through as_ptr's dispatch 3-4x that, on every
    per-tensor optimizer step), as_ptr for a list holding anything else."""
    try:
        ptrs = [x.data_ptr() for x in xs]
    except (AttributeError, TypeError):
        ptrs = [as_ptr(x) for x in xs]
    return _lib.ptr_array(ptrs)


class Stream:
    def __init__(self):
        s = C.c_void_p()
        check(lib().esgd_stream_create(C.byref(s)), "esgd_stream_create")
        self.handle = s.value

    def synchronize(self):
        check(lib().esgd_stream_synchronize(self.handle), "esgd_stream_synchronize")

    def close(self):
        if self.handle:
            lib().esgd_stream_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


class Event:
    def __init__(self):
        e = C.c_void_p()
        check(lib().esgd_event_create(C.byref(e)), "esgd_event_create")
        self.handle = e.value

    def record(self, stream=None):
        check(lib().esgd_event_record(self.handle, _sh(stream)), "esgd_event_record")

    def synchronize(self):
        check(lib().esgd_event_synchronize(self.handle), "esgd_event_synchronize")

    def elapsed_ms(self, stop: "Event") -> float:
        ms = C.c_float()
        check(lib().esgd_event_elapsed_ms(self.handle, stop.handle, C.byref(ms)), "elapsed")
        return float(ms.value)

    def close(self):
        if self.handle:
            lib().esgd_event_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def _sh(stream):
    if stream is None:
        return None
    return stream.handle if isinstance(stream, Stream) else int(stream)


class DeviceBuffer:
    """A device allocation of `count` elements of an esgd dtype."""

    def __init__(self, count: int, dtype: int = _lib.FLOAT):
        self.count, self.dtype = int(count), dtype
        self.nbytes = self.count * _lib.dtype_size(dtype)
        p = C.c_void_p()
        check(lib().esgd_malloc(C.byref(p), self.nbytes), "esgd_malloc")
        self.ptr = p.value

    def upload(self, arr: np.ndarray, stream=None, sync=True):
        arr = np.ascontiguousarray(arr, dtype=NP_DTYPE[self.dtype])
        assert arr.size == self.count, (arr.size, self.count)
        check(lib().esgd_memcpy_async(self.ptr, arr.ctypes.data, self.nbytes, 0, _sh(stream)), "h2d")
        if sync:
            synchronize(stream)
        return self

    def download(self, stream=None) -> np.ndarray:
        out = np.empty(self.count, dtype=NP_DTYPE[self.dtype])
        check(lib().esgd_memcpy_async(out.ctypes.data, self.ptr, self.nbytes, 1, _sh(stream)), "d2h")
        synchronize(stream)
        return out

    def zero(self, stream=None):
        check(lib().esgd_memset_async(self.ptr, 0, self.nbytes, _sh(stream)), "memset")

    def close(self):
        if self.ptr:
            lib().esgd_free(self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def synchronize(stream=None):
    if stream is None:
        check(lib().esgd_stream_synchronize(None), "esgd_stream_synchronize")
    else:
        check(lib().esgd_stream_synchronize(_sh(stream)), "esgd_stream_synchronize")


def device_synchronize():
    check(lib().esgd_device_synchronize(), "esgd_device_synchronize")


def reduce(dtype: int, inputs, out, count: int, stream=None, scale: float | None = None):
    """out = tree(inputs) on the device (esgd_reduce / esgd_reduce_scaled)."""
    ptrs = _lib.ptr_array([as_ptr(x) for x in inputs])
    if scale is None:
        rc = lib().esgd_reduce(dtype, len(inputs), ptrs, as_ptr(out), count, _sh(stream))
    else:
        rc = lib().esgd_reduce_scaled(dtype, len(inputs), ptrs, as_ptr(out), count, scale, _sh(stream))
    return check(rc, "esgd_reduce")


def reduce_host(dtype: int, inputs, out, count: int, stream=None):
    """out = tree(inputs) for HOST buckets (int addresses or numpy arrays; pinned ones
    move by async DMA): chunked H2D / tree kernel / D2H through HBM staging
    (esgd_reduce_host).  Stream-ordered: synchronize `stream` before reading `out`."""
    def hp(x):
        return x.ctypes.data if hasattr(x, "ctypes") else int(x)
    ptrs = _lib.ptr_array([hp(x) for x in inputs])
    return check(lib().esgd_reduce_host(dtype, len(inputs), ptrs, hp(out), count, _sh(stream)),
                 "esgd_reduce_host")


def vsum(dtype: int, a, b, c, count: int, stream=None):
    return check(lib().esgd_vsum(dtype, as_ptr(a), as_ptr(b), as_ptr(c), count, _sh(stream)), "esgd_vsum")


def pack_div(srcs, counts, dst, divisor: float = 1.0, stream=None):
    """dst = concat(src_i / divisor) (esgd_pack_div, fp32)."""
    n = len(srcs)
    c = (C.c_uint64 * max(1, n))(*[int(x) for x in counts])
    return check(lib().esgd_pack_div(n, ptr_array_of(srcs), c, as_ptr(dst),
                                     float(divisor), _sh(stream)), "esgd_pack_div")


def unpack(dsts, counts, src, stream=None):
    n = len(dsts)
    c = (C.c_uint64 * max(1, n))(*[int(x) for x in counts])
    return check(lib().esgd_unpack(n, ptr_array_of(dsts), c, as_ptr(src),
                                   _sh(stream)), "esgd_unpack")


def fill_uniform(buf: DeviceBuffer, seed: int, rank: int, stream=None):
    if buf.dtype == _lib.FLOAT:
        rc = lib().esgd_fill_uniform_f32(seed, rank, buf.ptr, buf.count, _sh(stream))
    elif buf.dtype == _lib.BF16:
        rc = lib().esgd_fill_uniform_bf16(seed, rank, buf.ptr, buf.count, _sh(stream))
    else:
        raise ValueError("fill_uniform: FLOAT or BF16 only")
    return check(rc, "esgd_fill_uniform")


def memory_stats() -> dict:
    """The bucket arena's footprint (esgd_memory_stats): bytes reserved from the driver,
    in use, and reserved in IPC-exported chunks."""
    r, u, x = C.c_uint64(), C.c_uint64(), C.c_uint64()
    check(lib().esgd_memory_stats(C.byref(r), C.byref(u), C.byref(x)), "esgd_memory_stats")
    return {"reserved": r.value, "in_use": u.value, "exported": x.value}
