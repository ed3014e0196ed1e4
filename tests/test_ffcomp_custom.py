"""ffcomp with a user operator (ffcomp_operator_create, F/src/ff.h:131-135): a host function
that the reference runs itself, on the host, over host buffers, once per post
(F/src/components/gcomp/ffop_gcomp.c:29-64; handles FFCUSTOM + i,
ffop_gcomp_operator.c:124-141).  libesgd does the same -- no GPU involved, so this runs on the
CPU -- and the answer is pinned by evaluation/custom_computation.c's c = a + b + 1 through the
oracle (ffref.comp_custom_plus_one, MIN of the three counts)."""
import ctypes as C

import numpy as np
import pytest

from conftest import LIB
from oracle import ffref

FFINT32, FFSUCCESS, FFINVALID_ARG, FFCUSTOM = 0, 0, -2, 6
ESGD_FF_DEVICE_BUFFERS = 1 << 20
OPFUN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int)


def _lib():
    lib = C.CDLL(LIB)
    vp = C.c_void_p
    lib.ffcomp_operator_create.argtypes = [OPFUN, C.c_int, C.POINTER(C.c_int)]
    lib.ffcomp_operator_delete.argtypes = [C.c_int]
    lib.ffcomp.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.POINTER(vp)]
    lib.ffbuffer_create.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
    lib.ffbuffer_delete.argtypes = [vp]
    lib.ffcomp_b.argtypes = [vp, vp, C.c_int, C.c_int, vp, C.POINTER(vp)]
    for f in ("ffop_post", "ffop_wait", "ffop_free"):
        getattr(lib, f).argtypes = [vp]
    lib.ffop_test.argtypes = [vp, C.POINTER(C.c_int)]
    return lib


@OPFUN
def plus_one(a, b, c, count, dtype):   # custom_computation.c:12-24
    if dtype != FFINT32:
        return FFINVALID_ARG
    ia = np.ctypeslib.as_array(C.cast(a, C.POINTER(C.c_int32)), (count,)) if count else np.zeros(0, np.int32)
    ib = np.ctypeslib.as_array(C.cast(b, C.POINTER(C.c_int32)), (count,)) if count else np.zeros(0, np.int32)
    ic = np.ctypeslib.as_array(C.cast(c, C.POINTER(C.c_int32)), (count,)) if count else np.zeros(0, np.int32)
    ic[:] = ia + ib + 1
    return FFSUCCESS


@OPFUN
def refuses(a, b, c, count, dtype):
    return -3


@pytest.mark.parametrize("na,nb,nc", [(1000, 1000, 1000), (1000, 700, 900), (17, 1000, 1000), (0, 5, 5)])
def test_user_operator_runs_on_host_buffers_with_min_counts(na, nb, nc):
    lib = _lib()
    h = C.c_int(-1)
    assert lib.ffcomp_operator_create(plus_one, 1, C.byref(h)) == FFSUCCESS
    assert h.value >= FFCUSTOM
    rng = np.random.default_rng(na * 7 + nb)
    a = rng.integers(-2**30, 2**30, na, dtype=np.int32)
    b = rng.integers(-2**30, 2**30, nb, dtype=np.int32)
    c = np.full(nc, -7, np.int32)
    bufs = [C.c_void_p() for _ in range(3)]
    for x, bh in zip((a, b, c), bufs):
        assert lib.ffbuffer_create(x.ctypes.data, len(x), FFINT32, 0, C.byref(bh)) == FFSUCCESS
    op = C.c_void_p()
    assert lib.ffcomp_b(bufs[0], bufs[1], h.value, 0, bufs[2], C.byref(op)) == FFSUCCESS
    assert lib.ffop_post(op) == FFSUCCESS and lib.ffop_wait(op) == FFSUCCESS
    flag = C.c_int(0)
    assert lib.ffop_test(op, C.byref(flag)) == FFSUCCESS and flag.value == 1
    lib.ffop_free(op)
    for bh in bufs:
        lib.ffbuffer_delete(bh)
    assert lib.ffcomp_operator_delete(h.value) == FFSUCCESS
    want = ffref.comp_custom_plus_one(a, b, nc)   # its c starts zeroed: compare the MIN prefix
    m = min(na, nb, nc)
    assert np.array_equal(c[:m], want[:m])
    assert np.all(c[m:] == -7)   # nothing written past MIN(counts)


def test_user_operator_handles_status_and_refusals():
    lib = _lib()
    count = 64
    a, b, c = (np.arange(count, dtype=np.int32) for _ in range(3))
    h1, h2 = C.c_int(), C.c_int()
    assert lib.ffcomp_operator_create(plus_one, 1, C.byref(h1)) == FFSUCCESS
    assert lib.ffcomp_operator_create(refuses, 0, C.byref(h2)) == FFSUCCESS
    assert h1.value != h2.value and min(h1.value, h2.value) >= FFCUSTOM
    op = C.c_void_p()
    # the function's status is the post's (ffop_gcomp.c:57-60)
    assert lib.ffcomp(a.ctypes.data, b.ctypes.data, count, FFINT32, h2.value, 0, c.ctypes.data, C.byref(op)) == 0
    assert lib.ffop_post(op) == -3
    lib.ffop_free(op)
    # a host function never runs on device buffers; unknown / deleted handles are refused
    assert lib.ffcomp(a.ctypes.data, b.ctypes.data, count, FFINT32, h1.value, ESGD_FF_DEVICE_BUFFERS,
                      c.ctypes.data, C.byref(op)) == FFINVALID_ARG
    assert lib.ffcomp_operator_delete(h2.value) == FFSUCCESS
    assert lib.ffcomp(a.ctypes.data, b.ctypes.data, count, FFINT32, h2.value, 0, c.ctypes.data,
                      C.byref(op)) == FFINVALID_ARG
    assert lib.ffcomp_operator_delete(h2.value) == FFINVALID_ARG
    assert lib.ffcomp_operator_create(C.cast(None, OPFUN), 1, C.byref(h2)) == FFINVALID_ARG
    # the freed slot is handed out again
    h3 = C.c_int()
    assert lib.ffcomp_operator_create(refuses, 0, C.byref(h3)) == FFSUCCESS and h3.value == h2.value
    lib.ffcomp_operator_delete(h3.value)
    lib.ffcomp_operator_delete(h1.value)


@OPFUN
def times_two(a, b, c, count, dtype):
    ic = np.ctypeslib.as_array(C.cast(c, C.POINTER(C.c_int32)), (count,)) if count else np.zeros(0, np.int32)
    ia = np.ctypeslib.as_array(C.cast(a, C.POINTER(C.c_int32)), (count,)) if count else np.zeros(0, np.int32)
    ic[:] = ia * 2
    return FFSUCCESS


def test_comp_keeps_its_operator_after_the_handle_is_deleted_and_reused():
    # the reference copies the operator into the op when the comp is made
    # (ffop_gcomp.c:9, ffop_gcomp_operator_get).  Deleting the handle afterwards -- and a new
    # ffcomp_operator_create taking the same slot -- must not change what the comp runs, nor
    # send it down the FFSUM path.
    lib = _lib()
    h = C.c_int(-1)
    assert lib.ffcomp_operator_create(plus_one, 1, C.byref(h)) == FFSUCCESS
    n = 64
    a = np.arange(n, dtype=np.int32)
    b = np.full(n, 10, np.int32)
    c = np.zeros(n, np.int32)
    op = C.c_void_p()
    assert lib.ffcomp(a.ctypes.data, b.ctypes.data, n, FFINT32, h.value, 0, c.ctypes.data, C.byref(op)) == FFSUCCESS
    assert lib.ffcomp_operator_delete(h.value) == FFSUCCESS
    h2 = C.c_int(-1)
    assert lib.ffcomp_operator_create(times_two, 1, C.byref(h2)) == FFSUCCESS
    assert h2.value == h.value                       # the slot was reused
    assert lib.ffop_post(op) == FFSUCCESS and lib.ffop_wait(op) == FFSUCCESS
    assert np.array_equal(c, ffref.comp_custom_plus_one(a, b, n))   # still a + b + 1
    lib.ffop_free(op)
    lib.ffcomp_operator_delete(h2.value)
