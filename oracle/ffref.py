"""ORACLE — numpy/ctypes front end of oracle/libffref.so (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product (eager-sgd_amd/) never does.  See oracle/ffref.h for the
reference file:line each routine restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(_HERE, "libffref.so")

INT32, INT64, DOUBLE, FLOAT = 0, 1, 2, 3
_NP = {INT32: np.int32, INT64: np.int64, DOUBLE: np.float64, FLOAT: np.float32}
_CODE = {np.dtype(v): k for k, v in _NP.items()}

_lib = None


def build():
    """Compile libffref.so with the reference's float flags (no fast-math)."""
    src = os.path.join(_HERE, "ffref.c")
    subprocess.check_call([
        "gcc", "-O3", "-ftree-vectorize", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
        "-shared", "-std=c11", "-o", SO, src, "-lpthread"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        h = C.CDLL(SO)
        vp, u32, i = C.c_void_p, C.c_uint32, C.c_int
        h.ffref_vsum.argtypes = [i, vp, vp, vp, u32]
        h.ffref_allreduce_rd.argtypes = [i, i, u32, C.POINTER(vp), C.POINTER(vp), vp]
        h.ffref_allreduce_rd_threads.argtypes = [i, i, u32, C.POINTER(vp), C.POINTER(vp),
                                                 C.POINTER(vp)]
        h.ffref_tree_sum.argtypes = [i, i, C.POINTER(vp), vp, u32]
        h.ffref_tree_sum_bf16.argtypes = [i, C.POINTER(vp), vp, u32]
        h.ffref_rand_r.argtypes = [C.POINTER(C.c_uint)]
        h.ffref_rand_r.restype = C.c_int
        h.ffref_fill_uniform_f32.argtypes = [C.c_uint64, i, vp, C.c_uint64]
        h.ffref_fill_uniform_f32_at.argtypes = [C.c_uint64, i, C.c_uint64, vp, C.c_uint64]
        h.ffref_splitmix64.argtypes = [C.c_uint64]
        h.ffref_splitmix64.restype = C.c_uint64
        h.ffref_f32_to_bf16.argtypes = [C.c_float]
        h.ffref_f32_to_bf16.restype = C.c_uint16
        h.ffref_time_allreduce.argtypes = [i, u32, i, i]
        h.ffref_time_allreduce.restype = C.c_double
        h.ffref_time_c1.argtypes = [i, u32, i, C.POINTER(i)]
        h.ffref_time_c1.restype = C.c_double
        h.ffref_time_c1_pinned.argtypes = [i, u32, i, C.POINTER(i), i, C.POINTER(i)]
        h.ffref_time_c1_pinned.restype = C.c_double
        _lib = h
    return _lib


def _code(a: np.ndarray) -> int:
    return _CODE[a.dtype]


def _pa(arrs):
    p = (C.c_void_p * len(arrs))()
    for j, a in enumerate(arrs):
        p[j] = a.ctypes.data
    return p


def vsum(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """c = a + b with the reference's FFSUM (ffop_gcomp_operator.c:33-58)."""
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    c = np.empty_like(a)
    rc = lib().ffref_vsum(_code(a), a.ctypes.data, b.ctypes.data, c.ctypes.data, a.size)
    assert rc == 0
    return c


def allreduce_rd(sendbufs, threads: bool = False):
    """Every rank's receive buffer after fflib2's recursive doubling
    (src/colls/ffallreduce.c:74-177), for P = len(sendbufs) simulated ranks."""
    sb = [np.ascontiguousarray(x) for x in sendbufs]
    P, n = len(sb), sb[0].size
    rb = [np.zeros_like(sb[0]) for _ in range(P)]
    if threads:
        tmp = [np.zeros_like(sb[0]) for _ in range(P)]
        rc = lib().ffref_allreduce_rd_threads(_code(sb[0]), P, n, _pa(sb), _pa(rb), _pa(tmp))
    else:
        scratch = np.zeros(P * n, dtype=sb[0].dtype)
        rc = lib().ffref_allreduce_rd(_code(sb[0]), P, n, _pa(sb), _pa(rb), scratch.ctypes.data)
    assert rc == 0
    return rb


def tree_sum(xs) -> np.ndarray:
    xs = [np.ascontiguousarray(x) for x in xs]
    out = np.empty_like(xs[0])
    assert lib().ffref_tree_sum(_code(xs[0]), len(xs), _pa(xs), out.ctypes.data, xs[0].size) == 0
    return out


def tree_sum_bf16(xs) -> np.ndarray:
    """bf16 bits in/out (uint16), fp32 tree accumulate, one RNE (extension, unpinned)."""
    xs = [np.ascontiguousarray(x, dtype=np.uint16) for x in xs]
    out = np.empty_like(xs[0])
    assert lib().ffref_tree_sum_bf16(len(xs), _pa(xs), out.ctypes.data, xs[0].size) == 0
    return out


def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    """Vectorised RNE f32 -> bf16 bits, same rule as ffref_f32_to_bf16."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    r = np.where(nan, ((u >> 16) | 0x40) & 0xFFFF, r)
    return r.astype(np.uint16)


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    return (np.asarray(h, dtype=np.uint32) << 16).view(np.float32)


def rand_r_sequence(seed: int, n: int):
    """glibc rand_r draws (restated), as used by ffrand_allreduce.c:88."""
    s = C.c_uint(seed)
    return [lib().ffref_rand_r(C.byref(s)) for _ in range(n)]


def activators(seed: int, P: int, n: int):
    """Majority activator of rounds 1..n: rand_r(&seed) % P (ffrand_allreduce.c:88)."""
    return [v % P for v in rand_r_sequence(seed, n)]


def fill_uniform(seed: int, rank: int, n: int, start: int = 0) -> np.ndarray:
    out = np.empty(n, dtype=np.float32)
    lib().ffref_fill_uniform_f32_at(seed, rank, start, out.ctypes.data, n)
    return out


def time_allreduce(P: int, count: int, threads: int, reps: int) -> float:
    return float(lib().ffref_time_allreduce(P, count, threads, reps))


def time_c1(P: int, count: int, reps: int, cpus=None):
    """(median seconds per step, every rank's result == tree) of the C1-shaped baseline:
    P ranks x (main + progress thread) (ffref.h: ffref_time_c1); cpus: 2P core ids, rank r's
    progress / main thread pinned to cpus[2r] / cpus[2r + 1] (ffref_time_c1_pinned)."""
    ok = C.c_int(0)
    if cpus:
        arr = (C.c_int * len(cpus))(*cpus)
        t = float(lib().ffref_time_c1_pinned(P, count, reps, arr, len(cpus), C.byref(ok)))
    else:
        t = float(lib().ffref_time_c1(P, count, reps, C.byref(ok)))
    return t, bool(ok.value)


_OPFUN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int)


def comp_custom_plus_one(a: np.ndarray, b: np.ndarray, nc: int) -> np.ndarray:
    """ffcomp with the user operator of evaluation/custom_computation.c:12-24
    (c = a + b + 1, int32) through the oracle's restatement of the gcomp backend's
    custom-operator call (ffref_comp_custom: size = MIN of the three counts,
    ffop_gcomp.c:29-56).  Returns the nc-element c (untouched elements stay 0)."""
    h = lib()
    a = np.ascontiguousarray(a, np.int32)
    b = np.ascontiguousarray(b, np.int32)
    c = np.zeros(nc, np.int32)
    fn = C.cast(h.ffref_op_plus_one, C.c_void_p).value
    comp = h.ffref_comp_custom
    comp.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p,
                     C.c_uint32]
    comp.restype = C.c_int
    rc = comp(fn, INT32, a.ctypes.data, a.size, b.ctypes.data, b.size, c.ctypes.data, nc)
    if rc != 0:
        raise RuntimeError(f"ffref_comp_custom: {rc}")
    return c
