/*
 * rtg_math.h — the reference platform's float transcendentals, restated bit for bit.
 *
 * The reference integrator calls acosf / sinf / cosf / atan2f from the C library
 * (RTBase/Sampling.h:35-61, RTBase/Core.h:549-557, RTBase/Lights.h:152-155). Path tracing turns a
 * 1-ulp difference in a sampled direction into a different path, so per-pixel
 * parity with the reference's own CPU render (BASELINE.json north_star) needs the *same* results
 * as the reference's libm, not merely accurate ones. The reference platform here is x86-64 Linux
 * with glibc 2.35 (this image and the GPU box). These functions restate glibc's published
 * algorithms, operation for operation, so the GPU kernels, the C oracle and the C++ host all
 * return exactly what glibc returns:
 *
 *   sinf, cosf, sincosf   glibc sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, s_sincosf.c,
 *                         sincosf.h, sincosf_data.c (Szabolcs Nagy's double-precision kernels:
 *                         one-step reduction below 120, 4/pi in 192 bits above). x86-64 glibc
 *                         selects its FMA build (__sinf_fma, ...) by ifunc on every CPU with
 *                         FMA + AVX2 (the build container's Xeon and the box's EPYC 9575F); the
 *                         kernels below use fma() exactly where that build's code does.
 *   acosf                 glibc sysdeps/ieee754/flt-32/e_acosf.c (fdlibm float, rational p/q)
 *   atan2f, atanf         glibc sysdeps/ieee754/flt-32/e_atan2f.c, s_atanf.c (fdlibm float)
 *
 * Exhaustive check (oracle/libm_check.c, test infrastructure): every one of the 2^32 float inputs
 * of sinf / cosf / sincosf / acosf, and 2^30 structured + random (y, x) pairs of atan2f, give the
 * bits of the host glibc (NaN payloads aside); profiles/r03_libm_exhaustive.txt. The GPU runs the
 * same code (tests/test_gpu_parity.py::test_device_math_matches_glibc).
 *
 * Rules that keep host and gfx950 identical:
 *   - float operations are IEEE binary32 with round-to-nearest-even; division and sqrtf are
 *     correctly rounded on both targets (gfx950: v_div_scale/fmas/fixup, refined v_sqrt);
 *   - fma() only where written (RTM_FMA: one rounding on both targets);
 *   - translation units that include this header MUST be compiled with -ffp-contract=off.
 *
 * Plain C99 so that the C oracle (oracle/), the C++ host and the HIP kernels share one definition.
 */
#ifndef RTG_MATH_H
#define RTG_MATH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define RTM_FN static inline __host__ __device__
#else
#define RTM_FN static inline
#endif

#define RTM_PI 3.1415926535897931 /* M_PI (binary64), used by the reference's fp64 islands */
#define RTM_FMA(a, b, c) __builtin_fma((a), (b), (c))

RTM_FN uint32_t rtm_asuint(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
RTM_FN float rtm_asfloat(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }

/* ------------------------------------------------------------------ sinf / cosf / sincosf
 * __sincosf_table[0] (sincosf_data.c). Table [1] is table [0] with the cosine coefficients negated;
 * with round-to-nearest every fma/mul of the cosine kernel is then exactly negated, so the kernels
 * below run on table [0] and negate the result instead. */
#define RTM_HPI_INV 0x1.45f306dc9c883p+23 /* 2/pi * 2^24 (no round-to-int intrinsic on x86-64) */
#define RTM_HPI 0x1.921fb54442d18p+0      /* pi/2 */
#define RTM_C0 0x1p0
#define RTM_C1 -0x1.ffffffd0c621cp-2
#define RTM_C2 0x1.55553e1068f19p-5
#define RTM_C3 -0x1.6c087e89a359dp-10
#define RTM_C4 0x1.99343027bf8c3p-16
#define RTM_S1 -0x1.555545995a603p-3
#define RTM_S2 0x1.1107605230bc4p-7
#define RTM_S3 -0x1.994eb3774cf24p-13
#define RTM_PI63 0x1.921fb54442d18p-62 /* 2 pi * 2^-64 */

/* sinf_poly / sincosf_poly, even (sine) branch: x3 = x*x2, s1 = fma(x2, S3, S2), x7 = x3*x2,
 * s = fma(x3, S1, x), result fma(s1, x7, s). */
RTM_FN double rtm_ksin(double x, double x2)
{
    const double x3 = x * x2;
    const double s1 = RTM_FMA(x2, RTM_S3, RTM_S2);
    const double x7 = x3 * x2;
    const double s = RTM_FMA(x3, RTM_S1, x);
    return RTM_FMA(s1, x7, s);
}
/* odd (cosine) branch: x4 = x2*x2, c1 = fma(x2, C1, C0), c2 = fma(x2, C4, C3), x6 = x4*x2,
 * c = fma(x4, C2, c1), result fma(c2, x6, c). */
RTM_FN double rtm_kcos(double x2)
{
    const double x4 = x2 * x2;
    const double c1 = RTM_FMA(x2, RTM_C1, RTM_C0);
    const double c2 = RTM_FMA(x2, RTM_C4, RTM_C3);
    const double x6 = x4 * x2;
    const double c = RTM_FMA(x4, RTM_C2, c1);
    return RTM_FMA(c2, x6, c);
}

/* reduce_large (sincosf.h): |y| >= 120 via a 32 x 96 -> 128-bit product with 4/pi (__inv_pio4). */
RTM_FN double rtm_reduce_large(uint32_t xi, int* np)
{
    const uint32_t inv_pio4[24] = {
        0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u, 0x6e4e4415u, 0x4e441529u,
        0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u, 0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u,
        0x34ddc0dbu, 0xddc0db62u, 0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
    const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * RTM_PI63;
}

/* The reduction shared by sinf / cosf / sincosf (s_sinf.c, s_cosf.c, s_sincosf.c), written as one
 * straight line for |y| < 120 (the GPU's lanes do not diverge): below pi/4 glibc skips the
 * reduction, but reduce_fast gives n = 0 there and x - 0 * hpi = x, so both branches are the same
 * operations; below 2^-12 the results are y and 1 (selected at the end). |y| >= 120 takes the
 * 192-bit reduction (m = n + sign, the large branch's sign[(n + sign) & 3] / table[(n + sign) & 2]).
 * Outputs: xs = the reduced argument times sign[m & 3] (the sine kernel's argument: the multiply by
 * +-1 is an exact negation), x2 = the square of the unsigned reduced argument (the cosine kernel's),
 * cneg = the cosine kernel runs on table [1] (m & 2), odd = n is odd (the kernels swap). */
typedef struct { double xs, x2; int cneg, odd; } rtm_sc_red;
RTM_FN rtm_sc_red rtm_sincos_reduce(float y)
{
    const uint32_t top = (rtm_asuint(y) >> 20) & 0x7ff;
    double x = (double)y;
    int n = 0, m;
    if (top < 0x42f) {  /* abstop12(y) < abstop12(120.0f): reduce_fast (TOINT_INTRINSICS = 0) */
        const double r = x * RTM_HPI_INV;
        n = ((int32_t)r + 0x800000) >> 24;
        x = RTM_FMA(-(double)n, RTM_HPI, x);  /* x - n * hpi (one vfnmadd in the FMA build) */
        m = n;
    } else if (top < 0x7f8) {
        const uint32_t xi = rtm_asuint(y);
        x = rtm_reduce_large(xi, &n);
        m = n + (int)(xi >> 31);
    } else {
        m = 0;  /* inf / NaN: the caller returns (y - y) / (y - y) */
    }
    rtm_sc_red o;
    o.x2 = x * x;
    o.xs = (((m + 1) & 2) != 0) ? -x : x;  /* sign[4] = {1, -1, -1, 1} */
    o.cneg = (m & 2) != 0;
    o.odd = n & 1;
    return o;
}
#define RTM_SC_TINY(top) ((top) < 0x398)      /* abstop12(y) < abstop12(0x1p-12f) */
#define RTM_SC_INVALID(top) ((top) >= 0x7f8)  /* inf or NaN */

/* sinf: n even -> sine kernel, n odd -> cosine kernel. */
RTM_FN float rtm_sinf(float y)
{
    const uint32_t top = (rtm_asuint(y) >> 20) & 0x7ff;
    const rtm_sc_red r = rtm_sincos_reduce(y);
    const double c = rtm_kcos(r.x2);
    const float v = (float)(r.odd ? (r.cneg ? -c : c) : rtm_ksin(r.xs, r.x2));
    return RTM_SC_INVALID(top) ? (y - y) / (y - y) : RTM_SC_TINY(top) ? y : v;
}
/* cosf: sinf_poly(x * s, x * x, p, n ^ 1): n even -> cosine kernel, n odd -> sine kernel. */
RTM_FN float rtm_cosf(float y)
{
    const uint32_t top = (rtm_asuint(y) >> 20) & 0x7ff;
    const rtm_sc_red r = rtm_sincos_reduce(y);
    const double c = rtm_kcos(r.x2);
    const float v = (float)(r.odd ? rtm_ksin(r.xs, r.x2) : (r.cneg ? -c : c));
    return RTM_SC_INVALID(top) ? (y - y) / (y - y) : RTM_SC_TINY(top) ? 1.0f : v;
}
/* sincosf: one reduction, both kernels, the quadrant swap of sincosf_poly as selects. glibc's
 * sincosf performs the same operations as its sinf and cosf; oracle/libm_check.c checks all three
 * against glibc on every input. */
RTM_FN void rtm_sincosf(float y, float* sn, float* cs)
{
    const uint32_t top = (rtm_asuint(y) >> 20) & 0x7ff;
    const rtm_sc_red r = rtm_sincos_reduce(y);
    const double s = rtm_ksin(r.xs, r.x2);
    const double c0 = rtm_kcos(r.x2);
    const double c = r.cneg ? -c0 : c0;
    float fs = (float)(r.odd ? c : s), fc = (float)(r.odd ? s : c);
    if (RTM_SC_TINY(top)) { fs = y; fc = 1.0f; }
    if (RTM_SC_INVALID(top)) { fs = (y - y) / (y - y); fc = fs; }
    *sn = fs;
    *cs = fc;
}

/* ------------------------------------------------------------------ acosf (e_acosf.c) */
#define RTM_ACOS_PI 0x1.921fb4p+1f      /* 0x40490fda */
#define RTM_ACOS_PIO2_HI 0x1.921fb4p+0f /* 0x3fc90fda */
#define RTM_ACOS_PIO2_LO 0x1.4442d0p-24f /* 0x33a22168 */
RTM_FN float rtm_acos_p(float z)
{
    const float pS0 = 0x1.555556p-3f, pS1 = -0x1.4d6120p-2f, pS2 = 0x1.9c1550p-3f, pS3 = -0x1.48228cp-5f,
                pS4 = 0x1.9efe08p-11f, pS5 = 0x1.23de10p-15f;
    return z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
}
RTM_FN float rtm_acos_q(float z)
{
    const float qS1 = -0x1.33a272p+1f, qS2 = 0x1.02ae5ap+1f, qS3 = -0x1.6066c2p-1f, qS4 = 0x1.3b8c5cp-4f;
    return 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
}
/* The three branches of __ieee754_acosf share p(z)/q(z); here z, the square root and the final
 * combination are selected, so the rational is evaluated once (the same operations on the same
 * operands as the branch that glibc takes). */
RTM_FN float rtm_acosf(float x)
{
    const int32_t hx = (int32_t)rtm_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    const int small = ix < 0x3f000000;  /* |x| < 0.5 */
    const float zs = x * x, zn = (1.0f + x) * 0.5f, zp = (1.0f - x) * 0.5f;
    const float z = small ? zs : (hx < 0 ? zn : zp);
    const float s = __builtin_sqrtf(z);
    const float r = rtm_acos_p(z) / rtm_acos_q(z);
    /* |x| < 0.5 */
    const float v_small = RTM_ACOS_PIO2_HI - (x - (RTM_ACOS_PIO2_LO - x * r));
    /* x < -0.5 */
    const float wn = r * s - RTM_ACOS_PIO2_LO;
    const float v_neg = RTM_ACOS_PI - 2.0f * (s + wn);
    /* x > 0.5 */
    const float df = rtm_asfloat(rtm_asuint(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float wp = r * s + c;
    const float v_pos = 2.0f * (df + wp);
    float v = small ? v_small : (hx < 0 ? v_neg : v_pos);
    if (small && ix <= 0x32800000) v = RTM_ACOS_PIO2_HI + RTM_ACOS_PIO2_LO;  /* |x| < 2^-26 */
    if (ix == 0x3f800000) v = hx > 0 ? 0.0f : RTM_ACOS_PI + 2.0f * RTM_ACOS_PIO2_LO;
    if (ix > 0x3f800000) v = (x - x) / (x - x);
    return v;
}

/* ------------------------------------------------------------------ atanf (s_atanf.c)
 * The four argument reductions are one division num / den with selected operands (the operations
 * of the branch glibc takes); the tables are selects. */
RTM_FN float rtm_atanf(float x)
{
    const float aT0 = 0x1.555556p-2f, aT1 = -0x1.99999ap-3f, aT2 = 0x1.24924ap-3f, aT3 = -0x1.c71c70p-4f,
                aT4 = 0x1.745cdcp-4f, aT5 = -0x1.3b0f2ap-4f, aT6 = 0x1.10d66ap-4f, aT7 = -0x1.dde2d6p-5f,
                aT8 = 0x1.97b4b2p-5f, aT9 = -0x1.2b4442p-5f, aT10 = 0x1.0ad3aep-6f;
    const int32_t hx = (int32_t)rtm_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    const float ax = __builtin_fabsf(x);
    /* id: -1 |x| < 0.4375, 0 < 11/16, 1 < 19/16, 2 < 2.4375, 3 otherwise */
    const int id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
    const float num = id == 0 ? 2.0f * ax - 1.0f : id == 1 ? ax - 1.0f : id == 2 ? ax - 1.5f : -1.0f;
    const float den = id == 0 ? 2.0f + ax : id == 1 ? ax + 1.0f : id == 2 ? 1.0f + 1.5f * ax : ax;
    const float t = id < 0 ? x : num / den;
    const float z = t * t;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const float hi = id == 0 ? 0x1.dac670p-2f : id == 1 ? 0x1.921fb4p-1f : id == 2 ? 0x1.f730bcp-1f : 0x1.921fb4p+0f;
    const float lo = id == 0 ? 0x1.586ed2p-28f : id == 1 ? 0x1.4442d0p-25f : id == 2 ? 0x1.281f68p-25f : 0x1.4442d0p-24f;
    const float zz = hi - ((t * (s1 + s2) - lo) - t);
    float v = id < 0 ? t - t * (s1 + s2) : (hx < 0 ? -zz : zz);
    if (ix < 0x31000000) v = x;  /* |x| < 2^-29 */
    if (ix >= 0x4c000000) {      /* |x| >= 2^25 */
        const float big = 0x1.921fb4p+0f + 0x1.4442d0p-24f;
        v = ix > 0x7f800000 ? x + x : (hx > 0 ? big : -0x1.921fb4p+0f - 0x1.4442d0p-24f);
    }
    return v;
}

/* ------------------------------------------------------------------ atan2f (e_atan2f.c)
 * The general case runs unconditionally and the special operands (NaN, zeros, infinities) override
 * it. glibc's x == 1 shortcut (return atanf(y)) needs no case of its own: y / 1 = y exactly, atanf
 * is odd (it negates its result for negative arguments) and the k > 60 value equals atanf(2^25+),
 * so the general case gives the same bits (libm_check covers x = +-1). */
RTM_FN float rtm_atan2f(float y, float x)
{
    const float tiny = 1.0e-30f, pi_o_4 = 0x1.921fb6p-1f, pi_o_2 = 0x1.921fb6p+0f, pi = 0x1.921fb6p+1f,
                pi_lo = -0x1.777a5cp-24f;
    const int32_t hx = (int32_t)rtm_asuint(x), hy = (int32_t)rtm_asuint(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);  /* 2 * sign(x) + sign(y) */
    const int32_t k = (iy - ix) >> 23;
    float z = rtm_atanf(__builtin_fabsf(y / x));
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    const float zn = rtm_asfloat(rtm_asuint(z) ^ 0x80000000u);
    float v = m == 0 ? z : m == 1 ? zn : m == 2 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
    const float half_pi = hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (iy == 0x7f800000) v = half_pi;
    if (ix == 0x7f800000) {
        const float q = iy == 0x7f800000 ? pi_o_4 : 0.0f;
        v = m == 0 ? q + tiny : m == 1 ? -q - tiny : m == 2 ? (iy == 0x7f800000 ? 3.0f * pi_o_4 : pi) + tiny
                                                            : (iy == 0x7f800000 ? -3.0f * pi_o_4 : -pi) - tiny;
        if (iy != 0x7f800000 && m <= 1) v = m == 0 ? 0.0f : -0.0f;
    }
    if (ix == 0) v = half_pi;
    if (iy == 0) v = m <= 1 ? y : (m == 2 ? pi + tiny : -pi - tiny);
    if (ix > 0x7f800000 || iy > 0x7f800000) v = x + y;
    return v;
}

#endif /* RTG_MATH_H */
