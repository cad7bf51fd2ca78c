"""include/rtg_math.h: the shared transcendentals are the correctly-rounded results (computed in
binary64 and rounded once) on large random samples, with C99 special cases."""
import ctypes as C

import numpy as np
import pytest

from oracle.pyoracle import lib


def _vec(fn, xs):
    return np.array([fn(float(x)) for x in xs], np.float32)


def test_acos_sin_cos_correctly_rounded():
    L = lib("rtm")
    rng = np.random.default_rng(0)
    r = rng.random(20000, dtype=np.float32)
    x = (2 * r - 1).astype(np.float32)
    assert np.array_equal(_vec(L.or_acosf, x), np.arccos(x.astype(np.float64)).astype(np.float32))
    ph = (2.0 * np.pi * r.astype(np.float64)).astype(np.float32)
    assert np.array_equal(_vec(L.or_sinf, ph), np.sin(ph.astype(np.float64)).astype(np.float32))
    assert np.array_equal(_vec(L.or_cosf, ph), np.cos(ph.astype(np.float64)).astype(np.float32))
    sq = np.sqrt(r).astype(np.float32)
    assert np.array_equal(_vec(L.or_acosf, sq), np.arccos(sq.astype(np.float64)).astype(np.float32))


def test_atan2_correctly_rounded_and_special_cases():
    L = lib("rtm")
    rng = np.random.default_rng(1)
    y = rng.normal(size=20000).astype(np.float32)
    x = rng.normal(size=20000).astype(np.float32)
    got = np.array([L.or_atan2f(float(a), float(b)) for a, b in zip(y, x)], np.float32)
    assert np.array_equal(got, np.arctan2(y.astype(np.float64), x.astype(np.float64)).astype(np.float32))
    for a, b in [(0.0, 0.0), (-0.0, 0.0), (0.0, -0.0), (-0.0, -0.0), (1.0, 0.0), (-1.0, -0.0), (0.0, -1.0),
                 (-0.0, -1.0), (np.inf, np.inf), (-np.inf, 1.0), (1.0, -np.inf)]:
        want = np.float32(np.arctan2(np.float64(a), np.float64(b)))
        got = np.float32(L.or_atan2f(a, b))
        assert got.tobytes() == want.tobytes(), (a, b)


def test_acos_domain():
    L = lib("rtm")
    assert np.isnan(L.or_acosf(1.0000001)) and np.isnan(L.or_acosf(float("nan")))
    assert L.or_acosf(1.0) == 0.0 and L.or_acosf(-1.0) == np.float32(np.pi)
    assert np.float32(L.or_sinf(-0.0)).tobytes() == np.float32(-0.0).tobytes()


def test_fused_sincos_is_bit_identical():
    """rtm_sincosf (one reduction, branch-free quadrant selects; what the device's
    spherical_to_world uses) returns the bits of rtm_sinf / rtm_cosf."""
    L = lib("rtm")
    rng = np.random.default_rng(2)
    x = np.concatenate([
        (rng.random(2_000_000) * 2 * np.pi).astype(np.float32),            # phi = 2 pi r2
        np.arccos(rng.random(1_000_000)).astype(np.float32),               # theta
        rng.normal(scale=50.0, size=500_000).astype(np.float32),
        np.array([0.0, -0.0, np.pi / 4, -np.pi / 4, 3 * np.pi / 4, np.inf, -np.inf, np.nan], np.float32),
    ])
    x = np.ascontiguousarray(x)
    assert L.or_sincos_mismatch(x.ctypes.data_as(C.POINTER(C.c_float)), len(x)) == 0
