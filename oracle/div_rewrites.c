/*
 * div_rewrites.c — TEST INFRASTRUCTURE ONLY. Exhaustive proof (all 2^32 float inputs) that the
 * device's multiplications by a precomputed reciprocal return the bits of the reference's
 * divisions by a constant, for the four divisions of the shading path where k_shade uses them
 * (raytracingrenderer_amd/csrc/device/rtg_dev.h, "division by a constant"):
 *
 *   pi_f      x / (float)M_PI              Colour / M_PI in BSDF::evaluate / sample
 *                                          (Materials.h:131, 140), float division
 *             == (float)((double)x * (1.0 / (double)(float)M_PI))
 *   pi_d      (float)((double)x / M_PI)    cosineHemispherePDF wi.z / M_PI (Sampling.h:52-56) and
 *                                          EnvironmentMap::evaluate's acosf(wi.y) / M_PI
 *                                          (Lights.h:153), in binary64
 *             == (float)((double)x * (1.0 / M_PI))
 *   twopi_d   (float)((double)x / (2.0 * M_PI))   EnvironmentMap::evaluate's u / (2 * M_PI) (Lights.h:152)
 *             == (float)((double)x * (1.0 / (2.0 * M_PI)))
 *
 * Any NaN matches any NaN. Prints one line per rewrite with the inputs checked and the mismatch
 * count (and the first mismatch); exit status 1 on any. `div_rewrites [stride]` checks every
 * stride-th input (default 1: all 2^32). Built by raytracingrenderer_amd/build.py (build_oracle,
 * gcc -O2 -ffp-contract=off -pthread) into oracle/_build/div_rewrites; tests/test_math.py runs it
 * on every 31st input and on all 2^32 inputs (~8 s on 8 threads); the full run is recorded in
 * profiles/r05_div_rewrites_exhaustive.txt.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NT 8
#define NR 3
static const char* NAMES[NR] = {"pi_f", "pi_d", "twopi_d"};

typedef struct {
    uint64_t lo, hi, stride, n, bad[NR];
    uint32_t first[NR];
} Job;

static float asf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t asu(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static int same(float a, float b) { return (a != a && b != b) || asu(a) == asu(b); }

static void* work(void* arg)
{
    Job* j = (Job*)arg;
    const float pif = (float)M_PI;
    const volatile double r_pif = 1.0 / (double)pif, r_pi = 1.0 / M_PI, r_2pi = 1.0 / (2.0 * M_PI);
    const double rp = r_pif, rq = r_pi, r2 = r_2pi;
    for (uint64_t i = j->lo; i < j->hi; i += j->stride) {
        const float x = asf((uint32_t)i);
        ++j->n;
        float want[NR], got[NR];
        want[0] = x / pif;
        got[0] = (float)((double)x * rp);
        want[1] = (float)((double)x / M_PI);
        got[1] = (float)((double)x * rq);
        want[2] = (float)((double)x / (2.0 * M_PI));
        got[2] = (float)((double)x * r2);
        for (int k = 0; k < NR; ++k)
            if (!same(want[k], got[k]) && j->bad[k]++ == 0) j->first[k] = (uint32_t)i;
    }
    return NULL;
}

int main(int argc, char** argv)
{
    Job jobs[NT];
    pthread_t th[NT];
    const uint64_t stride = argc > 1 ? strtoull(argv[1], NULL, 0) : 1;
    if (stride < 1) return 2;
    /* spans are multiples of the stride, so every stride-th input of the whole range is checked */
    const uint64_t span = ((1ull << 32) / NT + stride - 1) / stride * stride;
    for (int t = 0; t < NT; ++t) {
        memset(&jobs[t], 0, sizeof(Job));
        jobs[t].stride = stride;
        jobs[t].lo = span * t < (1ull << 32) ? span * t : (1ull << 32);
        jobs[t].hi = t == NT - 1 ? (1ull << 32) : (span * (t + 1) < (1ull << 32) ? span * (t + 1) : (1ull << 32));
        pthread_create(&th[t], NULL, work, &jobs[t]);
    }
    int any = 0;
    uint64_t bad[NR] = {0}, n = 0;
    uint32_t first[NR] = {0};
    for (int t = 0; t < NT; ++t) pthread_join(th[t], NULL);
    for (int t = 0; t < NT; ++t) n += jobs[t].n;
    for (int t = NT - 1; t >= 0; --t)
        for (int k = 0; k < NR; ++k) {
            if (jobs[t].bad[k]) first[k] = jobs[t].first[k];
            bad[k] += jobs[t].bad[k];
        }
    for (int k = 0; k < NR; ++k) {
        printf("%-8s inputs %llu mismatches %llu", NAMES[k], (unsigned long long)n, (unsigned long long)bad[k]);
        if (bad[k]) printf(" first 0x%08x", first[k]);
        printf("\n");
        any |= bad[k] != 0;
    }
    return any;
}
