"""The device's reproduction of the reference's sequential fp64 sums (lo_seqsum.h mono_seq_sum, used by the
reference-exact iteration-0 scale, IterativeClosestPointOptimizer.cpp:304-316: std::sort, std::accumulate, then the
(r - mean)^2 loop) against the plain sequential loop, bit for bit, on inputs chosen to break it: halfway ties, exact
powers of two, binade boundaries, zeros, huge dynamic range, subnormals, the largest single-workgroup size."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _seq(x):
    s = 0.0
    for v in x:
        s = s + float(v)
    return s


@pytest.fixture(scope="module")
def ctx():
    from lidar_odometry_amd import IterativeClosestPointOptimizer
    o = IterativeClosestPointOptimizer(max_points=1 << 14)
    yield o
    o.close()


def _dev_sum(o, x, sort):
    from lidar_odometry_amd import lib
    x = np.ascontiguousarray(x, np.float64)
    out = C.c_double(0.0)
    st = (C.c_longlong * 4)()
    rc = lib().lo_seq_sum_f64(o.ctx, x.ctypes.data_as(C.POINTER(C.c_double)), len(x), int(sort), C.byref(out), st)
    assert rc == 0, rc
    return out.value, list(st)


def _cases():
    rng = np.random.default_rng(7)
    yield "residuals", np.abs(rng.normal(0, 0.05, 3962))
    yield "uniform", rng.uniform(0, 1, 4096)
    yield "ties_1/64", np.round(rng.uniform(0, 1, 5000) * 64) / 64
    yield "powers_of_two", 2.0 ** rng.integers(-30, 3, 3000)
    yield "zeros_first", np.concatenate([np.zeros(300), np.abs(rng.normal(0, 1, 2000))])
    yield "all_zero", np.zeros(777)
    yield "single", np.array([0.3])
    yield "equal", np.full(4096, 0.1)
    yield "dynamic_range", 10.0 ** rng.uniform(-300, 10, 2000)
    yield "subnormal", np.concatenate([np.full(50, 5e-324), rng.uniform(0, 1e-310, 200), rng.uniform(0, 1, 100)])
    yield "max_size", np.abs(rng.normal(0, 1, 16384)) ** 3
    yield "near_binade", np.concatenate([np.full(1000, 2.0 ** -10) * (1 + 2.0 ** -52 * rng.integers(0, 4, 1000)),
                                         np.full(1000, 2.0 ** -11)])
    r = np.sort(np.abs(rng.normal(0, 0.05, 3500)))
    m = _seq(r) / len(r)
    yield "variance_terms", (r - m) * (r - m)


@pytest.mark.parametrize("sort", [1, 0])
def test_seq_sum_bitwise(ctx, sort):
    for name, x in _cases():
        ref = _seq(np.sort(x) if sort else x)
        got, st = _dev_sum(ctx, x, sort)
        assert np.float64(got).view(np.uint64) == np.float64(ref).view(np.uint64), (name, got, ref, st)


def test_seq_sum_is_mostly_parallel(ctx):
    """The KITTI-like case: a few dozen segment heads, no segment summed term by term."""
    x = np.abs(np.random.default_rng(3).normal(0, 0.05, 3962))
    _, st = _dev_sum(ctx, x, 1)
    assert 0 < st[0] < 200 and st[1] == 0, st


def _seq32(x):
    s = np.float32(0.0)
    for v in np.asarray(x, np.float32):
        s = np.float32(s + v)
    return s


def _dev_sum32(o, x):
    from lidar_odometry_amd import lib
    x = np.ascontiguousarray(x, np.float32)
    out = C.c_float(0.0)
    st = (C.c_longlong * 4)()
    rc = lib().lo_seq_sum_f32(o.ctx, x.ctypes.data_as(C.POINTER(C.c_float)), len(x), C.byref(out), st)
    assert rc == 0, rc
    return np.float32(out.value), list(st)


def _cases32():
    rng = np.random.default_rng(11)
    yield "random_walk", rng.normal(0, 1, 200_000)
    yield "drift", rng.normal(0.01, 1, 100_000)
    yield "positive", np.abs(rng.normal(0, 1, 50_000)) ** 2
    yield "ties_1/8", np.round(rng.normal(0, 1, 30_000) * 8) / 8            # exact cancellations, halfway ties
    yield "products", rng.normal(0, 1, 70_000) * rng.normal(0, 1, 70_000) * np.abs(rng.normal(0, 0.1, 70_000))
    yield "zeros_sparse", np.where(rng.uniform(0, 1, 40_000) < 0.8, 0.0, rng.normal(0, 1, 40_000))
    yield "leading_zero_chunks", np.concatenate([np.zeros(9000), rng.normal(0, 1, 9000)])
    yield "tiny_and_huge", np.concatenate([rng.normal(0, 1e-30, 5000), rng.normal(0, 1e20, 100), rng.normal(0, 1, 5000)])
    yield "single", np.array([-0.5])
    yield "empty", np.zeros(0)
    yield "negative_zeros", np.array([-0.0] * 9000 + [0.0] + [-0.0] * 5)
    yield "sign_flips", np.tile([1.0, -1.0], 20_000) + rng.normal(0, 1e-3, 40_000)   # a head at every term
    yield "grow_then_cancel", np.concatenate([rng.normal(5, 1, 500_000), rng.normal(-5, 1, 500_000)])
    yield "large_products", rng.normal(0, 1, 1_000_000) * rng.normal(0, 1, 1_000_000) * 0.01


def test_seq_sum_f32_bitwise(ctx):
    """The large-scan exact path's 43 running fp32 sums (signed terms: g, off-diagonal H) reproduced bit for bit."""
    for name, x in _cases32():
        x32 = np.asarray(x, np.float32)
        ref = _seq32(x32)
        got, st = _dev_sum32(ctx, x32)
        print(name, len(x32), "heads / term-by-term segments / term-by-term chunks / us:", st, flush=True)
        assert got.view(np.uint32) == ref.view(np.uint32), (name, got, ref, st)


def test_seq_sum_f32_mostly_parallel(ctx):
    """A 1M-term column of products (the C5 normal-equation terms' shape): a small fraction of the terms head a
    segment and almost none is summed term by term (the edge margin 2^-10 trades heads for a few hundred failed
    checks: kMwEdgeBits in lo_exact.hip)."""
    rng = np.random.default_rng(5)
    x = (rng.normal(0, 1, 1_000_000) * rng.normal(0, 1, 1_000_000) * 0.01).astype(np.float32)
    got, st = _dev_sum32(ctx, x)
    assert got.view(np.uint32) == _seq32(x).view(np.uint32)
    assert 0 < st[0] < 60_000 and st[1] < 1000 and st[2] == 0, st
