"""include/rtg_math.h restates the reference platform's float transcendentals (glibc 2.35's sinf /
cosf / sincosf, acosf, atan2f: the functions RTBase calls at Sampling.h:35-61, Core.h:549-557 and
Lights.h:152-155), so the GPU, the oracle and the reference's own build agree bit for bit.

The full check runs every 2^32 float input through oracle/libm_check (profiles/r03_libm_exhaustive.txt);
the CPU suite repeats it on every 31st input and on 2^24 atan2 pairs, against the C library of the
machine the tests run on."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLD
from oracle.pyoracle import BUILD, lib

CHECK = os.path.join(BUILD, "libm_check")


def _run_check(*args):
    r = subprocess.run([CHECK] + [str(a) for a in args], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if "inputs" in l]
    assert lines and all(l.split()[-1] == "0" for l in lines)
    return lines


def test_restatement_digest_is_pinned():
    """include/rtg_math.h's own outputs (no C library involved, so on any host) on every 127th float
    and 2^20 atan2f pairs equal the digests recorded where they matched glibc 2.35's FMA build bit
    for bit on every input (tests/golden/rtm_digest.json, profiles/r03_libm_exhaustive.txt)."""
    want = json.load(open(os.path.join(GOLD, "rtm_digest.json")))
    r = subprocess.run([CHECK, "digest", want["digests"]["stride"]], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    got = r.stdout.split()
    assert dict(zip(got[6::2], got[7::2])) == want["digests"]
    assert want["platform"] == {"glibc": "2.35", "fma": "1", "avx2": "1"}


@pytest.mark.host_glibc
def test_unary_functions_equal_glibc_on_every_31st_float():
    """sinf, cosf, sincosf (and glibc's sincosf against its own sinf/cosf, so a compiler that fuses
    the reference's sin/cos pairs changes nothing) and acosf: 138.5M inputs spread over all
    exponents, signs, denormals, infinities and NaN."""
    lines = _run_check("unary", 0, 0xFFFFFFFF, 31)
    assert any(l.startswith("acosf") for l in lines) and any(l.startswith("sincosf.cos") for l in lines)


@pytest.mark.host_glibc
def test_atan2_equals_glibc_on_structured_pairs():
    """atan2f on 2^24 pairs: random bit patterns, unit-vector components (EnvironmentMap::evaluate's
    inputs), close exponents, x = +-1 (glibc's atanf shortcut) and every special operand."""
    _run_check("atan2", 24)


def _eval(flavour, fn, x, nout):
    out = np.zeros(nout, np.float32)
    lib(flavour).or_math_eval(fn, x.ctypes.data_as(C.POINTER(C.c_float)), len(x) if fn != 4 else len(x) // 2,
                              out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def same_bits(a, b):
    """Bit equality with any NaN equal to any NaN (x86 and gfx950 NaN payloads differ)."""
    return np.array_equal(np.where(np.isnan(a), np.float32(np.nan), a).view(np.uint32),
                          np.where(np.isnan(b), np.float32(np.nan), b).view(np.uint32))


@pytest.mark.host_glibc
def test_oracle_flavours_agree_on_the_sampled_directions():
    """The oracle's two builds (liboracle_rtm: include/rtg_math.h, liboracle_libm: the C library)
    on the path's actual arguments: theta = acosf(sqrt(r1)), acosf(1 - 2 r1), phi = 2 pi r2 and
    unit-vector components for the environment lookup."""
    rng = np.random.default_rng(0)
    r = rng.random(1 << 20, dtype=np.float32)
    th = np.sqrt(r).astype(np.float32)
    ph = (2.0 * np.pi * r.astype(np.float64)).astype(np.float32)
    z = (1 - 2 * r).astype(np.float32)
    for fn, x, n in ((3, th, len(th)), (3, z, len(z)), (2, ph, 2 * len(ph)), (0, ph, len(ph)), (1, ph, len(ph))):
        assert same_bits(_eval("rtm", fn, x, n), _eval("libm", fn, x, n)), fn
    d = rng.normal(size=(1 << 19, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    yx = np.ascontiguousarray(d[:, [2, 0]].astype(np.float32)).reshape(-1)
    assert same_bits(_eval("rtm", 4, yx, len(d)), _eval("libm", 4, yx, len(d)))


@pytest.mark.host_glibc
def test_special_cases():
    L, G = lib("rtm"), lib("libm")
    for v in (0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 1.0000001, -1.0000001, 1e-30, -1e-30, 2 ** -26, 120.0, -120.0,
              1e30, float("inf"), float("-inf"), float("nan"), 3.4028235e38, 1.4e-45):
        for fn in ("or_acosf", "or_sinf", "or_cosf"):
            a, b = np.float32(getattr(L, fn)(v)), np.float32(getattr(G, fn)(v))
            assert same_bits(np.array([a]), np.array([b])), (fn, v, a, b)
    sp = [0.0, -0.0, 1.0, -1.0, float("inf"), float("-inf"), float("nan"), 1e-40, 3e38, 2.0 ** 70, 2.0 ** -70]
    for y in sp:
        for x in sp:
            a, b = np.float32(L.or_atan2f(y, x)), np.float32(G.or_atan2f(y, x))
            assert same_bits(np.array([a]), np.array([b])), (y, x, a, b)


@pytest.mark.parametrize("stride", [31, 1])
def test_division_rewrites_are_exact(stride):
    """k_shade computes x / (float)M_PI, (double)x / M_PI and (double)x / (2 M_PI) as products with
    the reciprocal (rtg_dev.h, "division by a constant"); oracle/div_rewrites checks that they return
    the division's bits on every stride-th float input; stride 1 is all 2^32 inputs (~8 s on 8
    threads; recorded in profiles/r05_div_rewrites_exhaustive.txt). Pure IEEE binary32/binary64
    arithmetic, so the result holds on any host."""
    exe = os.path.join(BUILD, "div_rewrites")
    r = subprocess.run([exe, str(stride)], capture_output=True, text=True, timeout=900)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if "inputs" in l]
    assert [l.split()[0] for l in lines] == ["pi_f", "pi_d", "twopi_d"]
    for l in lines:
        f = l.split()
        assert int(f[2]) == ((1 << 32) + stride - 1) // stride and f[4] == "0", l


def test_fused_sincos_is_bit_identical():
    """rtm_sincosf (one reduction, branch-free quadrant selects; what the device's
    spherical_to_world uses) returns the bits of rtm_sinf / rtm_cosf."""
    L = lib("rtm")
    rng = np.random.default_rng(2)
    x = np.concatenate([
        (rng.random(2_000_000) * 2 * np.pi).astype(np.float32),            # phi = 2 pi r2
        np.arccos(rng.random(1_000_000)).astype(np.float32),               # theta
        rng.normal(scale=50.0, size=500_000).astype(np.float32),
        rng.normal(scale=1e6, size=100_000).astype(np.float32),            # the 192-bit reduction
        np.array([0.0, -0.0, np.pi / 4, -np.pi / 4, 3 * np.pi / 4, np.inf, -np.inf, np.nan], np.float32),
    ])
    x = np.ascontiguousarray(x)
    assert L.or_sincos_mismatch(x.ctypes.data_as(C.POINTER(C.c_float)), len(x)) == 0
