"""Pin the CPU oracle (oracle/ffref.c) before trusting it.

The reference cannot be executed here, so the oracle is pinned by the
reference's own known-answer tests and by this host's libc:
  * evaluation/allreduce.c:59-63        reduced[j] == (i+j)*size after an int32 allreduce
  * evaluation/rsgd.c:87,100            inputs of 1.0 -> result counts the contributors
  * evaluation/solo_allreduce_correctness.c / rand_allreduce_correctness.c
                                        schedule result == plain allreduce of the inputs
  * glibc rand_r                        ffrand_allreduce.c:88's activator draw
and by structural properties of fflib2's recursive doubling (src/colls/ffallreduce.c).
"""
import ctypes
import ctypes.util
import json
import os

import numpy as np
import pytest

from oracle import ffref


def test_rand_r_matches_libc(golden_dir):
    with open(os.path.join(golden_dir, "rand_r.json")) as f:
        gold = json.load(f)["sequences"]
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    for seed, seq in gold.items():
        assert ffref.rand_r_sequence(int(seed), len(seq)) == seq
        s = ctypes.c_uint(int(seed))
        assert [libc.rand_r(ctypes.byref(s)) for _ in range(len(seq))] == seq


@pytest.mark.parametrize("P", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("it", [0, 5, 1000])
def test_known_answer_int32(P, it):
    # evaluation/allreduce.c:49-63: to_reduce[j] = i + j; expect (i + j) * size
    n = 3000
    x = [np.arange(it, it + n, dtype=np.int32) for _ in range(P)]
    for rb in ffref.allreduce_rd(x):
        np.testing.assert_array_equal(rb, (np.arange(n, dtype=np.int64) + it) * P)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_contributor_count(P):
    # evaluation/rsgd.c:87,100: every contributor writes 1.0, the rest 0.0
    n = 2048
    for present in range(P + 1):
        x = [np.full(n, 1.0 if r < present else 0.0, np.float32) for r in range(P)]
        for rb in ffref.allreduce_rd(x):
            assert np.all(rb == present)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_all_ranks_bit_identical_and_tree(P):
    rng = np.random.default_rng(P)
    x = [rng.standard_normal(10007).astype(np.float32) * np.float32(10.0 ** rng.integers(-3, 3)) for _ in range(P)]
    rbs = ffref.allreduce_rd(x)
    tree = ffref.tree_sum(x)
    for rb in rbs:  # commutativity of IEEE add -> every rank holds rank 0's tree
        assert rb.view(np.uint32).tolist() == tree.view(np.uint32).tolist()


def test_explicit_butterfly_p8():
    rng = np.random.default_rng(1)
    x = [rng.standard_normal(513).astype(np.float32) for _ in range(8)]
    f = np.float32
    want = ((x[1] + x[0]) + (x[3] + x[2])) + ((x[5] + x[4]) + (x[7] + x[6]))
    np.testing.assert_array_equal(ffref.tree_sum(x).view(np.uint32), want.astype(f).view(np.uint32))
    lin = x[0].copy()
    for r in range(1, 8):
        lin = lin + x[r]
    assert np.any(lin != want)  # order matters: a linear (ring) sum is not the reference


def test_non_power_of_two_partial_result():
    # ffallreduce.c:140 skips partners >= P: at P=3 rank 1 never sees x2
    x = [np.full(64, v, np.float32) for v in (1.0, 2.0, 4.0)]
    rb = ffref.allreduce_rd(x)
    assert np.all(rb[0] == 7) and np.all(rb[2] == 7) and np.all(rb[1] == 3)
    np.testing.assert_array_equal(ffref.tree_sum(x), rb[0])


@pytest.mark.parametrize("P", [2, 4, 8])
def test_threaded_equals_sequential(P):
    x = [ffref.fill_uniform(0x5EEDE56D, r, 40000) for r in range(P)]
    a = ffref.allreduce_rd(x)
    b = ffref.allreduce_rd(x, threads=True)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u.view(np.uint32), v.view(np.uint32))


@pytest.mark.parametrize("n", [0, 1, 3, 1023, 1024, 1025, 4097])
@pytest.mark.parametrize("dt", [np.float32, np.float64, np.int32, np.int64])
def test_vsum_strips(n, dt):
    rng = np.random.default_rng(n)
    a = (rng.standard_normal(n) * 1000).astype(dt)
    b = (rng.standard_normal(n) * 1000).astype(dt)
    np.testing.assert_array_equal(ffref.vsum(a, b), (a + b).astype(dt))


def test_int32_wraps():
    a = np.array([2 ** 31 - 1, -(2 ** 31)], np.int32)
    b = np.array([1, -1], np.int32)
    np.testing.assert_array_equal(ffref.vsum(a, b), np.array([-(2 ** 31), 2 ** 31 - 1], np.int32))


def test_special_values_ieee():
    x = [np.array([np.inf, np.inf, 0.0, -0.0, 1e-45], np.float32),
         np.array([1.0, -np.inf, -0.0, -0.0, 1e-45], np.float32)]
    out = ffref.tree_sum(x)
    assert out[0] == np.inf and np.isnan(out[1])
    assert out[2] == 0 and not np.signbit(out[2])          # 0 + -0 = +0
    assert out[3] == 0 and np.signbit(out[3])              # -0 + -0 = -0
    assert out[4] == 2 * np.finfo(np.float32).smallest_subnormal   # subnormals kept (no FTZ)


def test_bf16_rounding_rules():
    v = np.array([1.0, 1.00390625, 1.01171875, -2.5, np.inf, np.nan, 0.0, -0.0,
                  3.3895314e38, 1e-40], np.float32)
    h = ffref.f32_to_bf16(v)
    assert h[0] == 0x3F80 and h[1] == 0x3F80        # tie to even
    assert h[2] == 0x3F82                           # tie rounds up to even
    assert h[4] == 0x7F80 and (h[5] & 0x7F80) == 0x7F80 and (h[5] & 0x7F)
    assert h[6] == 0 and h[7] == 0x8000
    back = ffref.bf16_to_f32(h)
    assert np.isnan(back[5]) and back[3] == -2.5
    for i, f in enumerate(v):  # scalar C routine agrees with the vectorised one
        assert ffref.lib().ffref_f32_to_bf16(float(f)) == h[i]


def test_bf16_tree_error_bound():
    rng = np.random.default_rng(3)
    xf = rng.standard_normal((8, 5000)).astype(np.float32)
    xb = ffref.f32_to_bf16(xf)
    out = ffref.bf16_to_f32(ffref.tree_sum_bf16(list(xb)))
    exact = ffref.bf16_to_f32(xb).astype(np.float64).sum(0)
    # fp32 accumulation error is negligible next to the single bf16 rounding
    assert np.all(np.abs(out - exact) <= np.abs(exact) * 2 ** -8 + 1e-6)


def test_fill_uniform_range_and_determinism():
    a = ffref.fill_uniform(0x5EEDE56D, 3, 100000)
    b = ffref.fill_uniform(0x5EEDE56D, 3, 100000)
    c = ffref.fill_uniform(0x5EEDE56D, 4, 100000)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert a.min() >= -1 and a.max() < 1 and abs(a.mean()) < 0.01


@pytest.mark.parametrize("P", [2, 4, 8])
def test_golden_vectors_reproduce(golden_dir, P):
    g = np.load(os.path.join(golden_dir, f"tree_f32_p{P}.npz"))
    for name in ("gauss", "special"):
        rb = ffref.allreduce_rd(list(g[f"{name}_x"]))
        np.testing.assert_array_equal(np.stack(rb).view(np.uint32), g[f"{name}_rb"].view(np.uint32))


def test_golden_known_int32(golden_dir):
    g = np.load(os.path.join(golden_dir, "known_int32.npz"))
    for key in g.files:
        if key.endswith("_x"):
            x, rb = g[key], g[key[:-2] + "_rb"]
            P = x.shape[0]
            np.testing.assert_array_equal(rb, np.broadcast_to(x[0].astype(np.int64) * P, rb.shape))
            np.testing.assert_array_equal(np.stack(ffref.allreduce_rd(list(x))), rb)


def test_golden_bf16(golden_dir):
    g = np.load(os.path.join(golden_dir, "tree_bf16_p8.npz"))
    np.testing.assert_array_equal(ffref.tree_sum_bf16(list(g["x"])), g["out"])


@pytest.mark.parametrize("na,nb,nc", [(1000, 1000, 1000), (1023, 1500, 2000), (4097, 100, 4097), (0, 5, 5)])
def test_custom_operator_plus_one_known_answer(na, nb, nc):
    # SURVEY.md §8(c) pin 4: evaluation/custom_computation.c:53-74 fills a, b with rand()
    # and checks c[i] == a[i] + b[i] + 1 for the user operator of :12-24; the gcomp
    # backend calls it over MIN(counts) elements (ffop_gcomp.c:52-56).  Oracle-side only:
    # FFCUSTOM is not on the GPU path.
    rng = np.random.default_rng(na + nb + nc)
    a = rng.integers(0, 2**31 - 1, na, dtype=np.int64).astype(np.int32)   # rand()'s range
    b = rng.integers(0, 2**31 - 1, nb, dtype=np.int64).astype(np.int32)
    c = ffref.comp_custom_plus_one(a, b, nc)
    m = min(na, nb, nc)
    want = (a[:m].astype(np.int64) + b[:m].astype(np.int64) + 1).astype(np.uint32).view(np.int32)
    assert np.array_equal(c[:m], want)
    assert not c[m:].any()
