"""Parity of the HIP reduction (esgd_reduce / esgd_vsum) with the CPU oracle.

Bar: bit-exact for fp32/fp64/int32/int64 against oracle/ffref.c's restatement of
fflib2's recursive doubling (NaN compared as NaN); bf16 (an extension the reference
lacks, parity unpinned) bit-exact against the oracle's fp32-accumulate + single-RNE
convention.
"""
import os

import numpy as np
import pytest

from esgd import _lib
from esgd.device import DeviceBuffer, Stream, fill_uniform, reduce, synchronize, vsum
from oracle import ffref

pytestmark = pytest.mark.gpu

NP = {_lib.FLOAT: np.float32, _lib.DOUBLE: np.float64, _lib.INT32: np.int32, _lib.INT64: np.int64}
U = {np.dtype(np.float32): np.uint32, np.dtype(np.float64): np.uint64,
     np.dtype(np.int32): np.uint32, np.dtype(np.int64): np.uint64, np.dtype(np.uint16): np.uint16}


def bits_equal(a: np.ndarray, b: np.ndarray):
    assert a.shape == b.shape and a.dtype == b.dtype
    if a.dtype.kind == "f":
        na, nb = np.isnan(a), np.isnan(b)
        assert np.array_equal(na, nb), "NaN positions differ"
        a, b = np.where(na, 0, a).astype(a.dtype), np.where(nb, 0, b).astype(b.dtype)
    ua, ub = a.view(U[a.dtype]), b.view(U[b.dtype])
    bad = np.nonzero(ua != ub)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}: {a[bad[:5]]} vs {b[bad[:5]]}"


def gpu_reduce(xs, dtype, out_alias=False, offset=0, scale=None):
    n = xs[0].size
    bufs = [DeviceBuffer(n + offset, dtype) for _ in xs]
    for b, x in zip(bufs, xs):
        host = np.zeros(n + offset, dtype=x.dtype)
        host[offset:] = x
        b.upload(host)
    es = _lib.dtype_size(dtype)
    ins = [b.ptr + offset * es for b in bufs]
    if out_alias:
        out, optr = bufs[0], ins[0]
    else:
        out = DeviceBuffer(n + offset, dtype)
        optr = out.ptr + offset * es
    reduce(dtype, ins, optr, n, scale=scale)
    synchronize()
    return out.download()[offset:]


def rand_input(dt, k, n, seed):
    rng = np.random.default_rng(seed)
    if np.dtype(dt).kind == "f":
        return [(rng.standard_normal(n) * 10.0 ** rng.integers(-2, 3)).astype(dt) for _ in range(k)]
    info = np.iinfo(dt)
    return [rng.integers(info.min, info.max, n, dtype=dt, endpoint=True) for _ in range(k)]


@pytest.mark.parametrize("dtype", [_lib.FLOAT, _lib.DOUBLE, _lib.INT32, _lib.INT64])
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("n", [1, 5, 1023, 4099, 65536 + 3])
def test_reduce_matches_oracle(dtype, k, n):
    xs = rand_input(NP[dtype], k, n, seed=k * 1000 + n)
    bits_equal(gpu_reduce(xs, dtype), ffref.tree_sum(xs))


@pytest.mark.parametrize("P", [2, 4, 8])
def test_golden_every_rank(golden_dir, P):
    g = np.load(os.path.join(golden_dir, f"tree_f32_p{P}.npz"))
    for name in ("gauss", "special"):
        x, rb = g[f"{name}_x"], g[f"{name}_rb"]
        out = gpu_reduce(list(x), _lib.FLOAT)
        for r in range(P):  # the one device result equals every reference rank's buffer
            bits_equal(out, rb[r])


def test_golden_known_int32(golden_dir):
    g = np.load(os.path.join(golden_dir, "known_int32.npz"))
    for key in g.files:
        if key.endswith("_x"):
            out = gpu_reduce(list(g[key]), _lib.INT32)
            np.testing.assert_array_equal(out, g[key[:-2] + "_rb"][0])


@pytest.mark.parametrize("k", [2, 8])
def test_misaligned_and_inplace(k):
    xs = rand_input(np.float32, k, 10001, seed=7)
    want = ffref.tree_sum(xs)
    bits_equal(gpu_reduce(xs, _lib.FLOAT, offset=1), want)       # scalar path
    bits_equal(gpu_reduce(xs, _lib.FLOAT, out_alias=True), want)  # rb = tmp + rb style


def test_zero_count_is_noop():
    b = DeviceBuffer(4)
    reduce(_lib.FLOAT, [b.ptr, b.ptr], b.ptr, 0)
    synchronize()


@pytest.mark.parametrize("dtype", [_lib.FLOAT, _lib.INT32, _lib.DOUBLE, _lib.INT64])
def test_vsum_matches_ffsum(dtype):
    a, b = rand_input(NP[dtype], 2, 5003, seed=11)
    da, db, dc = (DeviceBuffer(5003, dtype).upload(a), DeviceBuffer(5003, dtype).upload(b),
                  DeviceBuffer(5003, dtype))
    vsum(dtype, da, db, dc, 5003)
    bits_equal(dc.download(), ffref.vsum(a, b))


def test_bf16_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "tree_bf16_p8.npz"))
    out = gpu_reduce(list(g["x"]), _lib.BF16)
    np.testing.assert_array_equal(out, g["out"])


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_bf16_matches_oracle(k):
    rng = np.random.default_rng(k)
    xs = [ffref.f32_to_bf16(rng.standard_normal(9001).astype(np.float32)) for _ in range(k)]
    xs[0][:8] = ffref.f32_to_bf16(np.array([np.nan, np.inf, -np.inf, 0, -0.0, 1e-39, 3e38, -3e38],
                                           np.float32))
    np.testing.assert_array_equal(gpu_reduce(xs, _lib.BF16), ffref.tree_sum_bf16(xs))


@pytest.mark.parametrize("dtype", [_lib.FLOAT, _lib.BF16])
def test_scaled_reduce(dtype):
    # opt_esgd_solo_imagenet_imbalance.py:40 divides by comm size; fused here as one
    # fp32 multiply after the tree (exact IEEE product, then storage rounding)
    rng = np.random.default_rng(5)
    xf = [rng.standard_normal(7777).astype(np.float32) for _ in range(8)]
    if dtype == _lib.BF16:
        xs = [ffref.f32_to_bf16(x) for x in xf]
        t = [ffref.bf16_to_f32(x) for x in xs]
        tree = ffref.tree_sum(t)
        want = ffref.f32_to_bf16(tree * np.float32(0.125))
    else:
        xs = xf
        want = ffref.tree_sum(xs) * np.float32(0.125)
    bits_equal(gpu_reduce(xs, dtype, scale=0.125), want)


def test_fill_uniform_bitwise():
    for rank in (0, 3, 7):
        b = DeviceBuffer(100003)
        fill_uniform(b, 0x5EEDE56D, rank)
        bits_equal(b.download(), ffref.fill_uniform(0x5EEDE56D, rank, 100003))


def test_full_size_c2_bitwise():
    """Config C2 at full size: 8 staged 64 MiB fp32 buckets -> 1, generated on device
    by the shared splitmix generator and checked element-for-element."""
    n, k, seed = 16 * 1024 * 1024, 8, 0x5EEDE56D
    s = Stream()
    bufs = [DeviceBuffer(n) for _ in range(k)]
    for r, b in enumerate(bufs):
        fill_uniform(b, seed, r, stream=s)
    out = DeviceBuffer(n)
    reduce(_lib.FLOAT, [b.ptr for b in bufs], out, n, stream=s)
    s.synchronize()
    got = out.download()
    xs = [ffref.fill_uniform(seed, r, n) for r in range(k)]
    bits_equal(got, ffref.tree_sum(xs))


def download_slice(buf, start, m):
    """Elements [start, start + m) of a float32 device buffer."""
    from esgd._lib import check, lib
    out = np.empty(m, np.float32)
    check(lib().esgd_memcpy_async(out.ctypes.data, buf.ptr + start * 4, m * 4, 1, None), "d2h")
    synchronize()
    return out


def test_reduce_beyond_int32_elements():
    """Buckets longer than 2^31 elements (8 GiB of fp32: 128 windowed launches, each inside
    the buffer descriptors' 32-bit range), checked against the oracle on a head, a middle
    slice across element 2^31, and the ragged tail."""
    n, k, seed, m = (1 << 31) + 5, 2, 0x5EED0B16, 1 << 20
    bufs = [DeviceBuffer(n) for _ in range(k)]
    for r, b in enumerate(bufs):
        fill_uniform(b, seed, r)
    out = DeviceBuffer(n)
    reduce(_lib.FLOAT, [b.ptr for b in bufs], out, n)
    synchronize()
    for start in (0, (1 << 31) - m + 4, n - m):   # the middle slice ends past element 2^31
        want = ffref.tree_sum([ffref.fill_uniform(seed, r, m, start=start) for r in range(k)])
        bits_equal(download_slice(out, start, m), want)


def test_full_size_gate_256mib_bitwise():
    """The 1-GPU gate shape of BASELINE.json: 8 x 256 MiB fp32 buckets, checked in full."""
    n, k, seed = 64 * 1024 * 1024, 8, 0x5EEDE56D
    s = Stream()
    bufs = [DeviceBuffer(n) for _ in range(k)]
    for r, b in enumerate(bufs):
        fill_uniform(b, seed, r, stream=s)
    out = DeviceBuffer(n)
    reduce(_lib.FLOAT, [b.ptr for b in bufs], out, n, stream=s)
    s.synchronize()
    got = out.download()
    del bufs
    xs = [ffref.fill_uniform(seed, r, n) for r in range(k)]
    bits_equal(got, ffref.tree_sum(xs))


def _download(buf, start, m, np_dtype):
    from esgd._lib import check, lib
    out = np.empty(m, np_dtype)
    es = out.itemsize
    check(lib().esgd_memcpy_async(out.ctypes.data, buf.ptr + start * es, m * es, 1, None), "d2h")
    synchronize()
    return out


@pytest.mark.parametrize("dtype,n", [(_lib.FLOAT, 25 * (1 << 20) + 3), (_lib.BF16, 56 * (1 << 20) + 5)])
def test_windowed_buckets_ragged(dtype, n):
    """Buckets above 96 MiB run as 64 MiB windows (launch_windows): 8 inputs of 100 MiB fp32
    / 112 MiB bf16 with a ragged count, checked at the head, across the first window
    boundary and at the tail."""
    k, seed, m = 8, 0x5EED0B17, 1 << 16
    bf = dtype == _lib.BF16
    bufs = [DeviceBuffer(n, dtype) for _ in range(k)]
    for r, b in enumerate(bufs):
        fill_uniform(b, seed, r)
    out = DeviceBuffer(n, dtype)
    reduce(dtype, [b.ptr for b in bufs], out, n)
    synchronize()
    window = (64 << 20) // (2 if bf else 4)
    for start in (0, window - m // 2, n - m):
        xs = [ffref.fill_uniform(seed, r, m, start=start) for r in range(k)]
        if bf:
            want = ffref.tree_sum_bf16([ffref.f32_to_bf16(x) for x in xs])
            np.testing.assert_array_equal(_download(out, start, m, np.uint16), want)
        else:
            bits_equal(_download(out, start, m, np.float32), ffref.tree_sum(xs))


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("dtype", [_lib.FLOAT, _lib.DOUBLE, _lib.INT32, _lib.INT64])
@pytest.mark.parametrize("k", [1, 3, 8])
def test_reduce_host_buckets(k, dtype, pinned):
    # esgd_reduce_host: host buckets in and out (the reference's contract); pinned ones are
    # reduced in place through their device views (zero-copy), pageable ones chunked
    # through HBM staging (16 MiB per input and chunk: 3 chunks, a ragged last one, staging
    # sets reused within the call and across calls)
    import ctypes as C

    from esgd._lib import check, lib
    from esgd.device import reduce_host
    dt = NP[dtype]
    n = (37 << 20) // np.dtype(dt).itemsize + 5
    xs = rand_input(dt, k, n, 1000 + k)
    held = []

    def host_array(x):
        if not pinned:
            return np.array(x, copy=True)
        p = C.c_void_p()
        check(lib().esgd_host_alloc(C.byref(p), x.nbytes))
        held.append(p.value)
        a = np.frombuffer((C.c_char * x.nbytes).from_address(p.value), dtype=x.dtype)
        a[:] = x
        return a

    try:
        ins = [host_array(x) for x in xs]
        out = host_array(np.zeros(n, dt))
        s = Stream()
        reduce_host(dtype, ins, out, n, stream=s)
        s.synchronize()
        want = ffref.tree_sum(xs) if k > 1 else xs[0]
        bits_equal(out.copy(), want)
        # again, out aliasing input 0, staging sets carried over from the call above
        reduce_host(dtype, ins, ins[0], n, stream=s)
        s.synchronize()
        bits_equal(ins[0].copy(), want)
    finally:
        for p in held:
            lib().esgd_host_free(p)


def test_reduce_host_bf16_and_tiny():
    from esgd.device import reduce_host
    for n in (1, 7, 4099):
        xs = [ffref.f32_to_bf16(ffref.fill_uniform(0x5EED, r, n)) for r in range(5)]
        out = np.zeros(n, np.uint16)
        reduce_host(_lib.BF16, xs, out, n)
        synchronize()
        assert np.array_equal(out, ffref.tree_sum_bf16(xs)), n


# ---- the bucket arena behind esgd_malloc / esgd_free ----------------------

def test_free_while_kernel_in_flight_keeps_hipfree_semantics():
    # esgd_free returns a block to the arena for reuse by the next esgd_malloc of its
    # size; like hipFree it must first let the work queued on the device finish, or a
    # reduction still writing the freed block clobbers its next owner's data
    from esgd.device import Stream, memory_stats  # noqa: F401
    n = (64 << 20) // 4
    ins = [DeviceBuffer(n) for _ in range(8)]
    for r, b in enumerate(ins):
        fill_uniform(b, 0x5EED, r)
    synchronize()
    s1, s2 = Stream(), Stream()
    victim = DeviceBuffer(n)
    old = victim.ptr
    for _ in range(20):   # ~2 ms of writes into `victim` on s1
        reduce(_lib.FLOAT, [b.ptr for b in ins], victim, n, stream=s1)
    victim.close()        # while they run
    held = []             # other free runs of this size may be handed out first
    fresh = DeviceBuffer(n)
    while fresh.ptr != old and len(held) < 16:
        held.append(fresh)
        fresh = DeviceBuffer(n)
    assert fresh.ptr == old, "the arena should hand the freed block out again"
    fill_uniform(fresh, 0xABCDEF, 3, stream=s2)
    s2.synchronize()
    s1.synchronize()
    bits_equal(fresh.download(), ffref.fill_uniform(0xABCDEF, 3, n))


def test_arena_growth_bounded_over_a_size_sweep():
    # large blocks are carved best-fit from free chunk space and coalesce when freed, so
    # a sweep over many distinct bucket sizes reserves about its peak, not the sum
    from esgd.device import memory_stats
    MiB = 1 << 20
    sizes = [3, 300, 17, 129, 64, 250, 5, 96, 200, 33, 280, 7, 150, 301, 2.5, 111]
    st0 = memory_stats()
    base = st0["reserved"]
    for mib in sizes:
        b = DeviceBuffer(int(mib * MiB) // 4)
        b.close()
    grew = memory_stats()["reserved"] - base
    assert grew <= 304 * MiB, grew / MiB   # one 302 MiB chunk (2 MiB granules): idle ones were given back
    # two live at once, then freed: the runs coalesce back into one reusable span
    a, b = DeviceBuffer(150 * MiB // 4), DeviceBuffer(150 * MiB // 4)
    a.close(); b.close()
    c = DeviceBuffer(300 * MiB // 4)
    c.close()
    st = memory_stats()
    assert st["reserved"] - base <= 304 * MiB, st
    assert st["in_use"] == st0["in_use"], (st0, st)


def test_a_reported_hip_failure_does_not_fail_the_next_launch():
    # HIP keeps a failed call's status in the thread's last-error slot until
    # hipGetLastError() reads it, and every launch here is checked with hipGetLastError():
    # a failure the library reported (or tolerated) must not resurface as the next,
    # unrelated launch's error (round 3: "esgd_fill_uniform: invalid argument" after a
    # tolerated teardown failure)
    import ctypes as C
    import esgd
    rc = esgd.lib().esgd_free(C.c_void_p(0x7ff0dead0000))   # not a device allocation
    assert rc != 0
    b = DeviceBuffer(4099)
    fill_uniform(b, 0x5EED, 1)
    synchronize()
    bits_equal(b.download(), ffref.fill_uniform(0x5EED, 1, 4099))


SWEEPS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "bin",
                      "libesgd_sweeps.so")


@pytest.mark.skipif(not os.path.exists(SWEEPS), reason="tools/bin/libesgd_sweeps.so not built (make sweeps)")
def test_sweep_variants_match_oracle():
    # every measurement-only variant of the tree kernel (tools/sweeps/reduce_sweeps.hip,
    # behind tools/sweep_reduce.py's numbers) computes the oracle's bits: 8 ragged fp32
    # buckets, each policy of the table, plain and forced-grid launches
    import ctypes as C
    sw = C.CDLL(SWEEPS)
    sw.esgd_sweep_reduce.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.c_void_p,
                                     C.c_uint64, C.c_void_p]
    sw.esgd_sweep_last_error.restype = C.c_char_p
    n, k = (1 << 20) + 4099, 8
    s = Stream()   # every step on ONE stream (the legacy null stream does not order with it)
    bufs = [DeviceBuffer(n) for _ in range(k)]
    for r, b in enumerate(bufs):
        fill_uniform(b, 0x5EEDE56D, r, stream=s)
    out = DeviceBuffer(n)
    want = ffref.tree_sum([ffref.fill_uniform(0x5EEDE56D, r, n) for r in range(k)])
    pa = (C.c_void_p * 8)(*[b.ptr for b in bufs])
    bad = []
    for pol in [-1] + list(range(0, 39)):
        for unroll, nt, grid in ((4, 1, 0), (2, 0, 1024)):
            if pol != 0 and (unroll, nt) != (4, 1):
                continue
            out.zero(stream=s)
            rc = sw.esgd_sweep_reduce(pol, unroll, nt, grid, pa, out.ptr, n, s.handle)
            assert rc == 0, (pol, sw.esgd_sweep_last_error())
            s.synchronize()
            if not np.array_equal(out.download(stream=s).view(np.uint32), want.view(np.uint32)):
                bad.append((pol, unroll, nt, grid))
    assert not bad, bad


@pytest.mark.parametrize("divisor", [1.0, 3.0, 8.0])
def test_pack_div_and_unpack_bitwise(divisor):
    # esgd_pack_div / esgd_unpack (the fused optimizer bucket): tensors of ragged sizes packed
    # at arbitrary element offsets (4-B accesses), at 16-B aligned ones (vector path: sizes
    # that are multiples of 4), tiles of 16 Ki elements and their ragged ends; the division
    # is IEEE (x / divisor, numpy float32), unpack returns every tensor's slice bit for bit
    from esgd.device import pack_div, unpack
    sizes = [1, 3, 17, 1000, 16384, 16385, 70001, 8, 262147, 5, 4096, 49152, 7]
    rng = np.random.default_rng(7)
    xs = [(rng.standard_normal(n) * 10.0 ** rng.integers(-3, 4)).astype(np.float32) for n in sizes]
    bufs = [DeviceBuffer(n) for n in sizes]
    for b, x in zip(bufs, xs):
        b.upload(x)
    bucket = DeviceBuffer(sum(sizes))
    pack_div(bufs, sizes, bucket, divisor)
    synchronize()
    want = np.concatenate([x / np.float32(divisor) for x in xs]).astype(np.float32)
    bits_equal(bucket.download(), want)
    outs = [DeviceBuffer(n) for n in sizes]
    unpack(outs, sizes, bucket)
    synchronize()
    for o, x in zip(outs, xs):
        bits_equal(o.download(), x / np.float32(divisor))
