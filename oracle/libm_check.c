/*
 * libm_check.c — TEST INFRASTRUCTURE ONLY. Checks include/rtg_math.h (the restatement of glibc's
 * sinf / cosf / sincosf / acosf / atan2f that the GPU kernels, the oracle and the host use) against
 * the C library of the machine it runs on, bit for bit (any NaN matches any NaN: x86 and gfx950
 * produce different NaN payloads, and the film comparisons treat NaN as a mask).
 *
 *   libm_check unary [first last [stride]]    sinf, cosf, sincosf (both outputs, and against
 *                                             glibc's own sinf/cosf) and acosf on every float
 *                                             bit pattern in [first, last] (default: all 2^32),
 *                                             or every stride-th one
 *   libm_check digest [stride]                 no C library call: FNV-1a digests of rtg_math.h's own
 *                                             outputs on every stride-th float (default 31) and
 *                                             2^20 splitmix64 atan2f pairs, plus the host's glibc
 *                                             version and FMA/AVX2 flags (tests/golden/rtm_digest.json
 *                                             pins the digests where glibc 2.35's FMA build matched)
 *   libm_check atan2 [log2_pairs]              atan2f on 2^k pairs (default 2^30): random bit
 *                                             patterns, unit-vector components (the reference's
 *                                             EnvironmentMap::evaluate inputs, Lights.h:152),
 *                                             pairs of close exponents, x = 1, and the special
 *                                             values (zeros, infinities, NaN, denormals)
 *
 * Build: gcc -O2 -mfma -ffp-contract=off -fno-builtin -pthread libm_check.c -lm (the -mfma only
 * makes fma() an instruction; the results are the same without it). Prints one line per function
 * with the number of inputs and mismatches, then the first mismatches; exit status 1 on any.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <gnu/libc-version.h>

#include "../include/rtg_math.h"

#define NT_MAX 64
static float (*volatile g_sinf)(float) = sinf;
static float (*volatile g_cosf)(float) = cosf;
static float (*volatile g_acosf)(float) = acosf;
static float (*volatile g_atan2f)(float, float) = atan2f;
static void (*volatile g_sincosf)(float, float*, float*) = sincosf;

static int same(float a, float b)
{
    if (a != a && b != b) return 1;
    return rtm_asuint(a) == rtm_asuint(b);
}

enum { F_SIN, F_COS, F_SINCOS_S, F_SINCOS_C, F_GLIBC_SINCOS, F_ACOS, F_ATAN2, F_N };
static const char* NAMES[F_N] = {"sinf", "cosf", "sincosf.sin", "sincosf.cos", "glibc sincosf==sinf/cosf",
                                 "acosf", "atan2f"};

typedef struct {
    int mode;
    uint64_t lo, hi;  /* unary: bit range [lo, hi); atan2: pair index range */
    uint64_t stride;
    uint64_t bad[F_N], n[F_N];
    uint32_t ex_in[F_N][2];
    float ex_got[F_N], ex_want[F_N];
} Job;

static void record(Job* j, int f, int ok, uint32_t a, uint32_t b, float got, float want)
{
    j->n[f]++;
    if (ok) return;
    if (j->bad[f]++ == 0) { j->ex_in[f][0] = a; j->ex_in[f][1] = b; j->ex_got[f] = got; j->ex_want[f] = want; }
}

static uint64_t splitmix(uint64_t* s)
{
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static float u01(uint64_t* s) { return (float)(splitmix(s) >> 40) * (1.0f / 16777216.0f); }

/* the (y, x) pair number i of the atan2 sample */
static void atan2_pair(uint64_t i, float* y, float* x)
{
    static const uint32_t special[] = {0x00000000u, 0x80000000u, 0x7f800000u, 0xff800000u, 0x7fc00000u,
                                       0x3f800000u, 0xbf800000u, 0x00000001u, 0x80000001u, 0x007fffffu,
                                       0x00800000u, 0x7f7fffffu, 0xff7fffffu, 0x3f000000u, 0x5d000000u,
                                       0x21800000u};
    uint64_t s = i * 0x2545f4914f6cdd1dull + 17;
    const uint64_t r = splitmix(&s);
    switch (i & 7) {
    case 0: case 1:  /* random bit patterns: every exponent */
        *y = rtm_asfloat((uint32_t)r);
        *x = rtm_asfloat((uint32_t)(r >> 32));
        break;
    case 2: case 3: case 4: {  /* unit-vector components (uniform sphere and cosine-hemisphere dirs) */
        const float z = 1.0f - 2.0f * u01(&s), ph = 6.2831855f * u01(&s);
        const float sr = sqrtf(fmaxf(0.0f, 1.0f - z * z));
        *y = z;
        *x = sr * cosf(ph);
        if (i & 8) { float t = *y; *y = *x; *x = t; }
        break;
    }
    case 5: {  /* close exponents with random mantissas and signs (the divide and the reduction) */
        const uint32_t e = 64 + (uint32_t)(r % 120);
        const int32_t d = (int32_t)((r >> 8) % 9) - 4;
        *y = rtm_asfloat((uint32_t)((r >> 16) & 0x807fffffu) | ((e + (uint32_t)d) << 23));
        *x = rtm_asfloat((uint32_t)((r >> 40) & 0x7fffffu) | ((uint32_t)(r >> 63) << 31) | (e << 23));
        break;
    }
    case 6:  /* x = +-1 exactly (atanf path), y anything */
        *y = rtm_asfloat((uint32_t)r);
        *x = (r >> 63) ? -1.0f : 1.0f;
        break;
    default:  /* a special value against a random or special partner */
        *y = rtm_asfloat(special[r % 16]);
        *x = (r >> 20) & 1 ? rtm_asfloat(special[(r >> 8) % 16]) : rtm_asfloat((uint32_t)(r >> 32));
        if ((r >> 21) & 1) { float t = *y; *y = *x; *x = t; }
        break;
    }
}

static void* work(void* arg)
{
    Job* j = (Job*)arg;
    if (j->mode == 0) {
        for (uint64_t b = j->lo; b < j->hi; b += j->stride) {
            const uint32_t u = (uint32_t)b;
            const float x = rtm_asfloat(u);
            const float gs = g_sinf(x), gc = g_cosf(x);
            float ms, mc, gss, gcc;
            record(j, F_SIN, same(rtm_sinf(x), gs), u, 0, rtm_sinf(x), gs);
            record(j, F_COS, same(rtm_cosf(x), gc), u, 0, rtm_cosf(x), gc);
            rtm_sincosf(x, &ms, &mc);
            record(j, F_SINCOS_S, same(ms, gs), u, 0, ms, gs);
            record(j, F_SINCOS_C, same(mc, gc), u, 0, mc, gc);
            g_sincosf(x, &gss, &gcc);
            record(j, F_GLIBC_SINCOS, same(gss, gs) && same(gcc, gc), u, 0, gss, gs);
            const float ga = g_acosf(x), ma = rtm_acosf(x);
            record(j, F_ACOS, same(ma, ga), u, 0, ma, ga);
        }
    } else {
        for (uint64_t i = j->lo; i < j->hi; ++i) {
            float y, x;
            atan2_pair(i, &y, &x);
            const float g = g_atan2f(y, x), m = rtm_atan2f(y, x);
            record(j, F_ATAN2, same(m, g), rtm_asuint(y), rtm_asuint(x), m, g);
        }
    }
    return NULL;
}

static uint64_t fnv(uint64_t h, float v)
{
    uint32_t b = v != v ? 0x7fc00000u : rtm_asuint(v);  /* any NaN hashes as the canonical one */
    for (int k = 0; k < 4; ++k) { h ^= (b >> (8 * k)) & 0xffu; h *= 0x100000001b3ull; }
    return h;
}

static int digest_mode(uint64_t stride)
{
    uint64_t hs = 0xcbf29ce484222325ull, hc = hs, hsc = hs, ha = hs, ht = hs;
    for (uint64_t i = 0; i < (1ull << 32); i += stride) {
        const float x = rtm_asfloat((uint32_t)i);
        float s, c;
        rtm_sincosf(x, &s, &c);
        hs = fnv(hs, rtm_sinf(x));
        hc = fnv(hc, rtm_cosf(x));
        hsc = fnv(fnv(hsc, s), c);
        ha = fnv(ha, rtm_acosf(x));
    }
    uint64_t z = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < (1 << 20); ++i) {
        uint64_t r = (z += 0x9e3779b97f4a7c15ull);
        r = (r ^ (r >> 30)) * 0xbf58476d1ce4e5b9ull;
        r = (r ^ (r >> 27)) * 0x94d049bb133111ebull;
        r ^= r >> 31;
        ht = fnv(ht, rtm_atan2f(rtm_asfloat((uint32_t)r), rtm_asfloat((uint32_t)(r >> 32))));
    }
    printf("glibc %s fma %d avx2 %d\n", gnu_get_libc_version(), __builtin_cpu_supports("fma") ? 1 : 0,
           __builtin_cpu_supports("avx2") ? 1 : 0);
    printf("stride %llu sinf %016llx cosf %016llx sincosf %016llx acosf %016llx atan2f %016llx\n",
           (unsigned long long)stride, (unsigned long long)hs, (unsigned long long)hc, (unsigned long long)hsc,
           (unsigned long long)ha, (unsigned long long)ht);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) { fprintf(stderr, "usage: %s unary [first last] | atan2 [log2_pairs] | digest [stride]\n", argv[0]); return 2; }
    if (strcmp(argv[1], "digest") == 0) return digest_mode(argc >= 3 ? strtoull(argv[2], 0, 0) : 31);
    const int mode = strcmp(argv[1], "atan2") == 0;
    uint64_t lo = 0, hi = 1ull << 32;
    uint64_t stride = 1;
    if (!mode && argc >= 4) { lo = strtoull(argv[2], 0, 0); hi = strtoull(argv[3], 0, 0) + 1; }
    if (!mode && argc >= 5) stride = strtoull(argv[4], 0, 0);
    if (stride < 1) stride = 1;
    if (mode) hi = 1ull << (argc >= 3 ? atoi(argv[2]) : 30);
    int nt = 8;
    const char* e = getenv("LIBM_CHECK_THREADS");
    if (e) nt = atoi(e);
    if (nt < 1) nt = 1;
    if (nt > NT_MAX) nt = NT_MAX;
    static Job jobs[NT_MAX];
    pthread_t th[NT_MAX];
    const uint64_t steps = (hi - lo + stride - 1) / stride;
    const uint64_t span = ((steps + nt - 1) / nt) * stride;
    for (int t = 0; t < nt; ++t) {
        memset(&jobs[t], 0, sizeof(Job));
        jobs[t].mode = mode;
        jobs[t].stride = mode ? 1 : stride;
        jobs[t].lo = lo + span * t;
        jobs[t].hi = jobs[t].lo + span < hi ? jobs[t].lo + span : hi;
        if (jobs[t].lo > hi) jobs[t].lo = hi;
        pthread_create(&th[t], NULL, work, &jobs[t]);
    }
    uint64_t bad[F_N] = {0}, n[F_N] = {0};
    for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
    int any = 0;
    for (int f = 0; f < F_N; ++f) {
        for (int t = 0; t < nt; ++t) { bad[f] += jobs[t].bad[f]; n[f] += jobs[t].n[f]; }
        if (!n[f]) continue;
        printf("%-26s inputs %llu mismatches %llu\n", NAMES[f], (unsigned long long)n[f], (unsigned long long)bad[f]);
        for (int t = 0; t < nt; ++t)
            if (jobs[t].bad[f]) {
                printf("  first: in 0x%08x 0x%08x got 0x%08x want 0x%08x\n", jobs[t].ex_in[f][0], jobs[t].ex_in[f][1],
                       rtm_asuint(jobs[t].ex_got[f]), rtm_asuint(jobs[t].ex_want[f]));
                break;
            }
        any |= bad[f] != 0;
    }
    return any;
}
