/*
 * rtg_math.h — portable, bit-reproducible transcendentals for the rtg path tracer.
 *
 * The reference integrator calls acosf / sinf / cosf / atan2f from the platform libm
 * (RTBase/Sampling.h:35-61, RTBase/Core.h:549-557, RTBase/Lights.h:152-155). Two libms
 * (glibc vs ROCm ocml, or glibc vs MSVC CRT) disagree in the last ulp on a fraction of
 * inputs, and path tracing amplifies a 1-ulp change into visibly different paths
 * (SURVEY.md §0.5). To make the GPU wavefront renderer and the CPU oracle produce
 * *identical* bits, both call the functions below instead of a libm.
 *
 * Implementation rules (what makes them reproducible):
 *   - float in, float out; every intermediate is IEEE binary64;
 *   - only +, -, *, / on doubles (correctly rounded on x86-64 SSE2 and on gfx950),
 *     plus the correctly-rounded float sqrtf used as a seed; no fma, no libm;
 *   - translation units that include this header MUST be compiled with
 *     -ffp-contract=off (hipcc and gcc both contract a*b+c into fma otherwise).
 * Accuracy: < 2 ulp of binary64 before the final rounding, so the float result is the
 * correctly-rounded value except for inputs whose exact result lies within ~1e-16
 * (relative) of a float rounding midpoint.
 *
 * This header is plain C99 so that the C oracle (oracle/), the C++ host and the HIP
 * kernels share one definition.
 */
#ifndef RTG_MATH_H
#define RTG_MATH_H

#if defined(__HIPCC__) || defined(__HIP__)
#define RTM_FN static inline __host__ __device__
#else
#define RTM_FN static inline
#endif

#define RTM_PI      3.1415926535897931
#define RTM_PI_2    1.5707963267948966
#define RTM_PI_4    0.78539816339744828
#define RTM_3PI_4   2.3561944901923448
/* pi/2 split for Cody-Waite reduction: hi part has 33 significant bits, so k*hi is exact. */
#define RTM_PIO2_HI 1.57079632673412561417e+00
#define RTM_PIO2_LO 6.07710050650619224932e-11
#define RTM_INV_PIO2 6.36619772367581382433e-01

RTM_FN int rtm_isnan_d(double x) { return x != x; }
RTM_FN double rtm_fabs_d(double x) { return x < 0.0 ? -x : x; }

/* sin(r), cos(r) for |r| <= ~pi/4 (Taylor to r^17 / r^18; truncation < 1e-19). */
RTM_FN double rtm_ksin(double r)
{
    double z = r * r;
    double p = -1.0 / 1307674368000.0 + z * (1.0 / 355687428096000.0);
    p = 1.0 / 6227020800.0 + z * p;
    p = -1.0 / 39916800.0 + z * p;
    p = 1.0 / 362880.0 + z * p;
    p = -1.0 / 5040.0 + z * p;
    p = 1.0 / 120.0 + z * p;
    p = -1.0 / 6.0 + z * p;
    return r + (r * z) * p;
}
RTM_FN double rtm_kcos(double r)
{
    double z = r * r;
    double p = 1.0 / 20922789888000.0 + z * (-1.0 / 6402373705728000.0);
    p = -1.0 / 87178291200.0 + z * p;
    p = 1.0 / 479001600.0 + z * p;
    p = -1.0 / 3628800.0 + z * p;
    p = 1.0 / 40320.0 + z * p;
    p = -1.0 / 720.0 + z * p;
    p = 1.0 / 24.0 + z * p;
    p = -0.5 + z * p;
    return 1.0 + z * p;
}

/* sin or cos of a double with |x| < 2^19 (the path tracer only feeds [0, 2*pi]). */
RTM_FN double rtm_sincos_d(double x, int want_cos)
{
    if (rtm_isnan_d(x) || rtm_fabs_d(x) > 1.0e300) return x - x; /* NaN (inf - inf) */
    if (x == 0.0) return want_cos ? 1.0 : x; /* keeps sin(-0) = -0 */
    double fk = x * RTM_INV_PIO2;
    int k = (int)(fk + (fk >= 0.0 ? 0.5 : -0.5));
    double dk = (double)k;
    double r = (x - dk * RTM_PIO2_HI) - dk * RTM_PIO2_LO;
    int q = (k + (want_cos ? 1 : 0)) & 3;
    double v;
    switch (q) {
    case 0: v = rtm_ksin(r); break;
    case 1: v = rtm_kcos(r); break;
    case 2: v = -rtm_ksin(r); break;
    default: v = -rtm_kcos(r); break;
    }
    return v;
}

/* sin and cos of one argument: one reduction, both kernels, then branch-free quadrant selects (no
 * lane divergence on the GPU). Bit-identical to rtm_sincos_d(x, 0) and rtm_sincos_d(x, 1): the same
 * operations on the same operands; only the choice of result is a select instead of a switch. */
RTM_FN void rtm_sincos2_d(double x, double* sn, double* cs)
{
    if (rtm_isnan_d(x) || rtm_fabs_d(x) > 1.0e300) { *sn = x - x; *cs = x - x; return; }
    if (x == 0.0) { *sn = x; *cs = 1.0; return; }
    double fk = x * RTM_INV_PIO2;
    int k = (int)(fk + (fk >= 0.0 ? 0.5 : -0.5));
    double dk = (double)k;
    double r = (x - dk * RTM_PIO2_HI) - dk * RTM_PIO2_LO;
    double s = rtm_ksin(r), c = rtm_kcos(r);
    int q = k & 3;
    /* sin: q = 0 s, 1 c, 2 -s, 3 -c;  cos = sin at quadrant q + 1 */
    double a = (q & 1) ? c : s;
    double b = (q & 1) ? s : c;
    *sn = (q & 2) ? -a : a;
    *cs = ((q + 1) & 2) ? -b : b;
}

/* atan for 0 <= t <= 1: nearest node c = j/8, atan(t) = atan(c) + atan((t-c)/(1+t*c)). */
RTM_FN double rtm_atan01(double t)
{
    const double atan_tab[9] = {
        0.0,
        0.12435499454676144, 0.24497866312686414, 0.35877067027057225,
        0.46364760900080609, 0.55859931534356244, 0.64350110879328437,
        0.71882999962162453, 0.78539816339744828 };
    int j = (int)(t * 8.0 + 0.5);
    if (j > 8) j = 8;
    double c = (double)j * 0.125;
    double u = (t - c) / (1.0 + t * c); /* |u| <= 1/16 */
    double z = u * u;
    double p = -1.0 / 15.0 + z * (1.0 / 17.0);
    p = 1.0 / 13.0 + z * p;
    p = -1.0 / 11.0 + z * p;
    p = 1.0 / 9.0 + z * p;
    p = -1.0 / 7.0 + z * p;
    p = 1.0 / 5.0 + z * p;
    p = -1.0 / 3.0 + z * p;
    return atan_tab[j] + (u + (u * z) * p);
}

/* atan2 with the C99 Annex F special cases (signed zeros, infinities). */
RTM_FN double rtm_atan2_d(double y, double x)
{
    if (rtm_isnan_d(x) || rtm_isnan_d(y)) return x + y;
    int ys = (y < 0.0) || (y == 0.0 && 1.0 / y < 0.0);
    int xs = (x < 0.0) || (x == 0.0 && 1.0 / x < 0.0);
    double ay = ys ? -y : y;
    double ax = xs ? -x : x;
    double big = __builtin_inf();
    double r;
    if (ay == 0.0) {
        r = xs ? RTM_PI : 0.0;
    } else if (ax == 0.0) {
        r = RTM_PI_2;
    } else if (ax == big || ay == big) {
        if (ax == big && ay == big) r = xs ? RTM_3PI_4 : RTM_PI_4;
        else if (ax == big) r = xs ? RTM_PI : 0.0;
        else r = RTM_PI_2;
    } else {
        /* (ay <= ax) ? atan01(ay / ax) : pi/2 - atan01(ax / ay), with one division and one
         * atan01 (operand selects instead of two divergent branches) */
        int lo = ay <= ax;
        double at = rtm_atan01((lo ? ay : ax) / (lo ? ax : ay));
        double base = lo ? at : RTM_PI_2 - at;
        r = xs ? RTM_PI - base : base;
    }
    return ys ? -r : r;
}

/* sqrt of a double 0 <= a <= 4 seeded by the correctly-rounded float sqrt and refined by two
 * Newton steps in binary64 (deterministic: only + and / on doubles). */
RTM_FN double rtm_sqrt_d(double a)
{
    if (a <= 0.0) return a == 0.0 ? a : (a - a) / (a - a);
    float af = (float)a;
    double s = (double)__builtin_sqrtf(af); /* correctly rounded on both targets */
    s = 0.5 * (s + a / s);
    s = 0.5 * (s + a / s);
    return s;
}

RTM_FN double rtm_acos_d(double x)
{
    if (rtm_isnan_d(x)) return x + x;
    if (x > 1.0 || x < -1.0) return (x - x) / (x - x); /* NaN */
    double a = (1.0 - x) * (1.0 + x);
    return rtm_atan2_d(rtm_sqrt_d(a), x);
}

/* ---- float API (drop-in for the libm calls on the reference hot path) ---- */
RTM_FN float rtm_sinf(float x) { return (float)rtm_sincos_d((double)x, 0); }
RTM_FN float rtm_cosf(float x) { return (float)rtm_sincos_d((double)x, 1); }
RTM_FN void rtm_sincosf(float x, float* sn, float* cs)
{
    double s, c;
    rtm_sincos2_d((double)x, &s, &c);
    *sn = (float)s;
    *cs = (float)c;
}
RTM_FN float rtm_acosf(float x) { return (float)rtm_acos_d((double)x); }
RTM_FN float rtm_atan2f(float y, float x) { return (float)rtm_atan2_d((double)y, (double)x); }

#endif /* RTG_MATH_H */
