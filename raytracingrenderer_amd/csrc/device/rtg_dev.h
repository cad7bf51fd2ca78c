// rtg_dev.h — device data layout and reference-faithful device math for the wavefront tracer.
//
// Every helper here restates an RTBase expression with the same IEEE operation order
// (this TU is compiled with -ffp-contract=off; gfx950 f32 '/' and sqrtf are correctly rounded):
//   Vec3/Colour ops         RTBase/Core.h:16-195
//   Frame                   RTBase/Core.h:507-542
//   Ray::init               RTBase/Geometry.h:21-26 (invDir = 1/dir)
//   AABB::rayAABB           RTBase/Geometry.h:159-184 (Min/Max ternaries, std::max/min)
//   Triangle::rayIntersect  RTBase/Geometry.h:89-105 (plane test)
//   Texture::sample         RTBase/Imaging.h:72-94 (bilinear, integer wrap)
//   SamplingDistributions   RTBase/Sampling.h:44-69 (binary64 islands around M_PI)
//   fresnelDielectric       RTBase/Materials.h:55-77
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/rtg_math.h"

#define RTG_D __device__ __forceinline__
#define RTG_FLT_MAX 3.40282347e+38f
#define RTG_EPS 1e-4f                    // EPSILON, Geometry.h:60
#define RTG_PI_F 3.14159274f             // (float)M_PI, as in Colour / M_PI (Materials.h:131)
#define RTG_EXIT ((int)0x80000000)       // traversal sentinel (never a valid child word)
#define RTG_LEAF_SPAN 4                  // leaf word = ~(first triangle * RTG_LEAF_SPAN + count - 1)

namespace rtgd {

struct v3 { float x, y, z; };
RTG_D v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
RTG_D v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RTG_D v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RTG_D v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
RTG_D v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
RTG_D v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
RTG_D v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
RTG_D float dot(v3 a, v3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
RTG_D v3 cross(v3 a, v3 b) {
    return mk((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
RTG_D float length_sq(v3 a) { return ((a.x * a.x) + (a.y * a.y)) + (a.z * a.z); }
RTG_D v3 normalize(v3 a) {
    float l = 1.0f / sqrtf(((a.x * a.x) + (a.y * a.y)) + (a.z * a.z));
    return mk(a.x * l, a.y * l, a.z * l);
}
RTG_D float lum(v3 c) { return ((0.2126f * c.x) + (0.7152f * c.y)) + (0.0722f * c.z); }
// windows.h max/min macro semantics used by Renderer.h (max(NaN, 0) -> 0)
RTG_D float wmax(float a, float b) { return a > b ? a : b; }
RTG_D float wmin(float a, float b) { return a < b ? a : b; }
// std::max / std::min (libstdc++): max(a,b) = (a < b) ? b : a ; min(a,b) = (b < a) ? b : a
RTG_D float smax(float a, float b) { return (a < b) ? b : a; }
RTG_D float smin(float a, float b) { return (b < a) ? b : a; }

struct frame { v3 u, v, w; };
RTG_D frame frame_from(v3 n) {  // Frame::fromVector
    frame f;
    f.w = normalize(n);
    if (fabsf(f.w.x) > fabsf(f.w.y)) {
        float l = 1.0f / sqrtf(f.w.x * f.w.x + f.w.z * f.w.z);
        f.u = mk(f.w.z * l, 0.0f, -f.w.x * l);
    } else {
        float l = 1.0f / sqrtf(f.w.y * f.w.y + f.w.z * f.w.z);
        f.u = mk(0.0f, f.w.z * l, -f.w.y * l);
    }
    f.v = cross(f.w, f.u);
    return f;
}
RTG_D v3 to_local(const frame& f, v3 a) { return mk(dot(a, f.u), dot(a, f.v), dot(a, f.w)); }
RTG_D v3 to_world(const frame& f, v3 a) {
    return add(add(muls(f.u, a.x), muls(f.v, a.y)), muls(f.w, a.z));
}

// ------------------------------------------------------------------ device scene layout
// Internal BVH2 node, child-pair form: both child boxes live in the parent so one 64-byte fetch
// (4 x dwordx4) tests both. Child word: >= 0 internal node index; < 0 leaf, ~c = start*2 + (n-1).
struct __align__(16) DevNode {
    float4 a;  // lmin.x lmin.y lmin.z lmax.x
    float4 b;  // lmax.y lmax.z rmin.x rmin.y
    float4 c;  // rmin.z rmax.x rmax.y rmax.z
    int4 d;    // left word, right word, -, -
};
// Compressed 4-wide node (64 B). Slot boxes are stored conservatively: 8-bit offsets from the
// node's min corner in power-of-two steps, rounded outward and checked on the host with the
// device's own decode arithmetic, so a decoded box always contains the exact one. Exactness then
// rests on the leaf: a candidate hit counts only if its reference leaf box passes the exact slab
// test (leafbox, per triangle), which by containment also implies every ancestor's.
//   q[0] = origin.xyz, biased exponents (x | y<<8 | z<<16)
//   q[1] = planes min x, min y, min z, max x  (byte k = slot k)
//   q[2] = planes max y, max z, child words 0, 1
//   q[3] = child words 2, 3, -, -
// (A 48-B form and a 32-B form with 4-bit planes were measured slower: DESIGN.md §4.)
struct __align__(16) DevNodeQ {
    float4 q[4];
};
typedef float f2 __attribute__((ext_vector_type(2)));  // packed FP32 pair (v_pk_fma/mul/add_f32)
__host__ __device__ inline float qdecode(float origin, unsigned plane, int k, float scale) {
    return origin + (float)((plane >> (8 * k)) & 255u) * scale;
}
// Compact intersection record (48 B, three dwordx4 loads): n and the three vertices. d, e1, e2
// and invArea are recomputed with Triangle::init's own float ops (Geometry.h:72-83), so they are
// the same bits as a record that stores them.
struct __align__(16) DevTri48 {
    float4 a;  // n.xyz, v0.x
    float4 b;  // v0.yz, v1.xy
    float4 c;  // v1.z, v2.xyz
};
// Cold shading record (64 B): vertex normals, uvs, material.
struct __align__(16) DevShade {
    float4 a;  // n0.xyz n1.x
    float4 b;  // n1.yz n2.xy
    float4 c;  // n2.z u0 v0 u1
    float4 d;  // v1 u2 v2 material(int bits)
};
struct __align__(16) DevMat {
    int kind, two_sided, tex, is_light;
    float int_ior, ext_ior;
    int tex_wh;  // the albedo texture's width | height << 16; `tex` is its first texel in SceneView::texels
    int uniform;  // 1: every texel of the texture has the same bits (a 1x1 texture, or a constant one):
                  // bilinear() takes texel0 for its four taps instead of fetching them (same operands)
    float4 emission;
    float4 texel0;  // the texture's first texel (RGB)
};
struct __align__(16) DevLight {
    float4 v0a;  // v0.xyz, area       (area light)
    float4 v1t;  // v1.xyz, type bits  (0 area, 1 environment)
    float4 v2;   // v2.xyz, 1.0f / area (Triangle::sample's pdf, divided on the host)
    float4 gn;   // gNormal.xyz        (Triangle::gNormal)
    float4 em;   // emission rgb
};
struct DevTex { int off, w, h, pad; };

struct DevCamera {
    float ip[16];  // inverse projection
    float cm[16];  // camera
    float ox, oy, oz, width, height;
};

struct SceneView {
    const DevNode* nodes;    // reference BVH2 (rays with a zero direction component)
    const DevNodeQ* nodesq;  // compressed 4-wide tree (exact for rays with finite nonzero 1/d)
    const float4* leafbox;   // [2 per triangle] exact box of the reference leaf holding it
    const DevTri48* tris48;  // triangles (Triangle::rayIntersect's operands)
    const DevShade* shade;
    const DevMat* mats;
    const DevLight* lights;
    const DevTex* texinfo;
    const float4* texels;  // RGB + pad per texel
    int n_mats;          // distinct material records (prepare_scene merges identical ones)
    int n_lights;
    float pmf;           // 1.f / (float)n_lights, Scene::sampleLight's pmf, divided on the host
    int env_tex;         // -1: BackgroundColour(0)
    int env_off, env_w, env_h;  // the environment texture (first texel, size), kernel-argument copies
    int env_uniform;     // 1: every texel of the environment map has the same bits (env_one)
    float env_one[3];    // its first texel
    int root_word;       // child word of the root (RTG_EXIT if no triangles)
    int root_wordw;      // root word in the wide tree
    int usew;            // wide tree available (finite bounds, children inside parents)
    float root_box[6];   // bounds of the reference root node
    float cull_scale;    // scene magnitude used for the conservative cull inflation
    // small scenes (the wide nodes, triangle records and leaf boxes fit RTG_SMALL_F4 float4s, e.g.
    // the cornell box of config C2): one image [wide nodes | triangles | leaf boxes] that k_trace
    // copies into LDS per block, so every record fetch of the walk is an LDS read
    const float4* img;   // null: the walk reads global memory
    int img_n4, img_tri, img_lb;  // image size and the float4 offsets of the triangles / leaf boxes
};

// ------------------------------------------------------------------ Texture::sample
// texel fetchers: packed RGB (3 floats) or the device layout (RGB + pad, one 16-B load)
struct Texels3 {
    const float* t;
    RTG_D v3 operator()(int i) const { return mk(t[i * 3 + 0], t[i * 3 + 1], t[i * 3 + 2]); }
};
struct Texels4 {
    const float4* t;
    RTG_D v3 operator()(int i) const { const float4 v = t[i]; return mk(v.x, v.y, v.z); }
};
template <class TX>
RTG_D v3 bilinear(TX texel, int w, int h, float tu, float tv, bool uni = false, v3 one = v3{0.0f, 0.0f, 0.0f}) {
    float au = fabsf(tu), av = fabsf(tv);
    float u = smax(0.0f, au) * (float)w;
    float v = smax(0.0f, av) * (float)h;
    int x = (int)floorf(u);
    int y = (int)floorf(v);
    float fu = u - (float)x;
    float fv = v - (float)y;
    float w0 = (1.0f - fu) * (1.0f - fv);
    float w1 = fu * (1.0f - fv);
    float w2 = (1.0f - fu) * fv;
    float w3 = fu * fv;
    // x, y >= 0 here (u, v are >= 0 or +inf), so the modulo runs only when the coordinate wraps
    // and (x + 1) % w is a compare: same values as the reference's x % w, (x + 1) % w
    v3 s0, s1, s2, s3;
    if (uni) {  // every texel has the same bits (a 1x1 texture, or a constant one): the caller holds them
        s0 = s1 = s2 = s3 = one;
    } else {
        x = x < w ? x : x % w;
        y = y < h ? y : y % h;
        const int x1 = (x + 1 == w) ? 0 : x + 1, y1 = (y + 1 == h) ? 0 : y + 1;
        s0 = texel(y * w + x);
        s1 = texel(y * w + x1);
        s2 = texel(y1 * w + x);
        s3 = texel(y1 * w + x1);
    }
    return add(add(add(muls(s0, w0), muls(s1, w1)), muls(s2, w2)), muls(s3, w3));
}
// A material carries its texture's offset and size, and the environment's are kernel arguments, so
// the texels are one dependent fetch after the material record (no texinfo lookup between).
RTG_D v3 tex_sample(const SceneView& s, const DevMat& M, float tu, float tv) {
    return bilinear(Texels4{s.texels + M.tex}, M.tex_wh & 0xffff, (int)((unsigned)M.tex_wh >> 16), tu, tv,
                    M.uniform != 0, mk(M.texel0.x, M.texel0.y, M.texel0.z));
}

// ------------------------------------------------------------------ division by a constant
// The reference divides by M_PI in float (Colour / M_PI, Materials.h:131, 140) and in binary64
// (wi.z / M_PI, Sampling.h:52-56; u / (2 * M_PI) and acosf(wi.y) / M_PI, Lights.h:152-153). A
// binary64 product with the reciprocal, rounded to float, gives the same bits for every one of the
// 2^32 float inputs (oracle/div_rewrites.c, checked in tests/test_math.py): a few cycles instead of
// a correctly rounded division sequence (v_div_scale / rcp / fma / div_fmas / div_fixup).
RTG_D float div_pi_f(float x) { return (float)((double)x * (1.0 / (double)RTG_PI_F)); }  // x / (float)M_PI
RTG_D float div_pi_d(float x) { return (float)((double)x * (1.0 / RTM_PI)); }            // (float)((double)x / M_PI)
RTG_D float div_2pi_d(float x) { return (float)((double)x * (1.0 / (2.0 * RTM_PI))); }   // (float)((double)x / (2 M_PI))
RTG_D v3 divs_pi(v3 a) { return mk(div_pi_f(a.x), div_pi_f(a.y), div_pi_f(a.z)); }       // divs(a, (float)M_PI)

// ------------------------------------------------------------------ sampling (Sampling.h)
RTG_D v3 spherical_to_world(float theta, float phi) {  // Core.h:547-550
    float st, ct, sp, cp;  // rtm_sincosf: bit-identical to rtm_sinf / rtm_cosf
    rtm_sincosf(theta, &st, &ct);
    rtm_sincosf(phi, &sp, &cp);
    return mk(cp * st, sp * st, ct);
}
RTG_D v3 cosine_sample_hemisphere(float r1, float r2) {
    float theta = rtm_acosf(sqrtf(r1));
    float phi = (float)((2.0 * RTM_PI) * (double)r2);  // 2.0f * M_PI * r2 in binary64
    return spherical_to_world(theta, phi);
}
RTG_D v3 uniform_sample_sphere(float r1, float r2) {
    float theta = rtm_acosf(1.0f - 2.0f * r1);
    float phi = (float)((2.0 * RTM_PI) * (double)r2);
    return spherical_to_world(theta, phi);
}
RTG_D float uniform_sphere_pdf() { return (float)(1.0 / (4.0 * RTM_PI)); }

// EnvironmentMap::evaluate (Lights.h:150-157)
RTG_D v3 env_eval(const SceneView& s, v3 wi) {
    float u = rtm_atan2f(wi.z, wi.x);
    u = (u < 0.0f) ? (float)((double)u + 2.0 * RTM_PI) : u;
    u = div_2pi_d(u);                // (float)((double)u / (2.0 * M_PI))
    float v = div_pi_d(rtm_acosf(wi.y));  // (float)((double)acosf(wi.y) / M_PI)
    return bilinear(Texels4{s.texels + s.env_off}, s.env_w, s.env_h, u, v, s.env_uniform != 0,
                    mk(s.env_one[0], s.env_one[1], s.env_one[2]));
}
RTG_D v3 background(const SceneView& s, v3 dir) {
    if (s.env_tex < 0) return mk(0.0f, 0.0f, 0.0f);  // BackgroundColour(0,0,0)::evaluate
    return env_eval(s, dir);
}

// fresnelDielectric (Materials.h:55-77); returns R, writes wt when not TIR.
RTG_D float fresnel_dielectric(float cos_i, float ior_int, float ior_ext, v3& wt, v3 wol) {
    float ior = ior_int / ior_ext;
    float sin_i = sqrtf(1 - (cos_i * cos_i));
    float sin_t = ior * sin_i;
    float ior2sin2 = (ior * ior) * (1 - (cos_i * cos_i));
    if (ior2sin2 > 1.0f) return 1.0f;
    float cos_t = sqrtf(1 - (sin_t * sin_t));
    wt = mk(-ior * wol.x, -ior * wol.y, -cos_t);
    float fpa = (cos_i - ior * cos_t) / (cos_i + ior * cos_t);
    float fpe = (ior * cos_i - cos_t) / (ior * cos_i + ior * cos_t);
    float avg = ((fpa * fpa) + (fpe * fpe)) * 0.5f;
    return smax(0.0f, smin(1.0f, avg));  // clamp(avg, 0, 1) = max(0, min(1, avg))
}

// ------------------------------------------------------------------ RNG
RTG_D uint32_t pcg_step(uint64_t& s, uint64_t inc) {
    uint64_t old = s;
    s = old * 6364136223846793005ull + inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
}
RTG_D uint64_t pcg_inc(uint32_t pixel, uint32_t sample) {
    uint64_t seq = ((uint64_t)pixel << 16) | (uint64_t)sample;
    return (seq << 1u) | 1u;
}
RTG_D uint64_t pcg_seed(uint64_t seed, uint64_t inc) {
    uint64_t s = 0;
    pcg_step(s, inc);
    s += seed;
    pcg_step(s, inc);
    return s;
}
RTG_D float pcg_next(uint64_t& s, uint64_t inc) {
    return (float)(pcg_step(s, inc) >> 8) * (1.0f / 16777216.0f);
}

// Sampler adaptors: the path's PCG stream, or a scripted list (probe / unit tests).
struct PcgSampler {
    uint64_t s;
    uint64_t inc;
    RTG_D float next() { return pcg_next(s, inc); }
};
struct ScriptSampler {
    const float* v;
    int n, i;
    RTG_D float next() { return i < n ? v[i++] : 0.5f; }
};

// BSDF::sample for the three effective behaviours (Materials.h:127-134, 167-177, 218-226, 265-294,
// 335-343, 380-388, 433-441). alb = albedo->sample(tu, tv). Returns wi (world); writes
// reflectedColour and pdf. Draw order: Lambert family cosineSampleHemisphere(next(), next()) with
// g++'s right-to-left argument evaluation (first draw -> r2); glass draws only when R != 1.
template <class S>
RTG_D v3 bsdf_sample(int kind, float int_ior, float ext_ior, v3 alb, const frame& fr, v3 wo, S& smp,
                     v3& refl, float& pdf) {
    if (kind == 0 || kind == 1) {  // RTG_MAT_DIFFUSE / RTG_MAT_LAMBERT
        const float q2 = smp.next();
        const float q1 = smp.next();
        const v3 wl = cosine_sample_hemisphere(q1, q2);
        if (kind == 0) pdf = (wl.z >= 0.0f) ? div_pi_d(wl.z) : 0.0f;  // cosineHemispherePDF
        else pdf = div_pi_d(wl.z);                                      // stubs: wi.z / M_PI
        refl = divs_pi(alb);
        return to_world(fr, wl);
    }
    const v3 wol = to_local(fr, wo);
    if (kind == 2) {  // RTG_MAT_MIRROR
        pdf = 1.0f;
        refl = alb;
        return to_world(fr, mk(-wol.x, -wol.y, wol.z));
    }
    // RTG_MAT_GLASS
    const float cos_i = fabsf(wol.z);
    const bool enter = wol.z > 0.0f;
    const float eta_i = enter ? ext_ior : int_ior;
    const float eta_t = enter ? int_ior : ext_ior;
    v3 wt = mk(0.0f, 0.0f, 0.0f);
    const float R = fresnel_dielectric(cos_i, eta_i, eta_t, wt, wol);
    if (!enter) wt.z = -wt.z;
    const bool refl_dir = (R == 1.0f) || (smp.next() < R);
    v3 wi;
    if (refl_dir) {
        wi = mk(-wol.x, -wol.y, wol.z);
        pdf = R;
        refl = muls(alb, R);
    } else {
        wi = wt;
        pdf = 1.0f - R;
        refl = muls(alb, 1.0f - R);
    }
    return to_world(fr, wi);
}

// BSDF::PDF of the non-specular kinds: cosineHemispherePDF(shadingData.frame.toLocal(wi))
// (Materials.h:136-140, 227-232, 349-354, 394-399, 447-452; Sampling.h:52-56). Only z of toLocal is used.
RTG_D float bsdf_pdf_lambert(const frame& fr, v3 wi) {
    const float z = dot(wi, fr.w);
    return (z >= 0.0f) ? div_pi_d(z) : 0.0f;
}
// RayTracer::convertPDFAreaToSolidAngle / balanceHeuristic (Renderer.h:411-422)
RTG_D float pdf_area_to_solid(float pdf_area, float dist2, float cos_theta) {
    return cos_theta > 0.0f ? (pdf_area * dist2) / cos_theta : 0.0f;
}
RTG_D float balance_heuristic(float pa, float pb) { return pa / (pa + pb); }

// ------------------------------------------------------------------ intersection
// AABB::rayAABB with the reference's exact arithmetic; returns pass/fail.
RTG_D bool slab_exact(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, v3 o, v3 inv) {
    float ax = (mnx - o.x) * inv.x, ay = (mny - o.y) * inv.y, az = (mnz - o.z) * inv.z;
    float bx = (mxx - o.x) * inv.x, by = (mxy - o.y) * inv.y, bz = (mxz - o.z) * inv.z;
    float ex = ax < bx ? ax : bx, ey = ay < by ? ay : by, ez = az < bz ? az : bz;  // Min
    float xx = ax > bx ? ax : bx, xy = ay > by ? ay : by, xz = az > bz ? az : bz;  // Max
    float te = smax(smax(ex, ey), ez);
    float tx = smin(smin(xx, xy), xz);
    return !(tx < te || tx < 0);
}
// Conservative entry distance of the box inflated by delta (position space). Used only to
// skip boxes that cannot contain a hit closer than the current one; never to accept.
RTG_D float slab_cull_entry(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                            v3 o, v3 inv, float delta) {
    float nx = (inv.x >= 0.0f ? mnx - delta : mxx + delta);
    float ny = (inv.y >= 0.0f ? mny - delta : mxy + delta);
    float nz = (inv.z >= 0.0f ? mnz - delta : mxz + delta);
    float cx = (nx - o.x) * inv.x, cy = (ny - o.y) * inv.y, cz = (nz - o.z) * inv.z;
    return fmaxf(fmaxf(cx, cy), cz);  // fmaxf drops NaN -> conservative
}

// Triangle::rayIntersect on the 48-B record (Geometry.h:89-105). `want(t)` rejects a plane
// distance that cannot be a candidate for the caller (beyond the current hit or not in front):
// those never produce output, so the rest of the test (edge functions, 1/area) is skipped for them.
// The same test on the record in memory: n and v0 (the first 32 B, two dwordx4) decide t, and the
// last 16 B (v1.z, v2) are loaded as one aligned dwordx4 only when t is a candidate (left to
// itself the compiler re-loaded part of the second dwordx4 and split the third one in two).
template <class W>
RTG_D bool tri_intersect48p(const DevTri48* P, v3 o, v3 d, W want, float& t, float& u, float& v, unsigned& tails) {
    const float4 A = P->a, B = P->b;
    const v3 n = mk(A.x, A.y, A.z);
    const float denom = dot(n, d);
    if (denom == 0) return false;
    const v3 v0 = mk(A.w, B.x, B.y);
    const float dd = dot(n, v0);
    const float tt = (dd - dot(n, o)) / denom;
    if (tt < 0 || !want(tt)) return false;
    ++tails;  // (counting builds only: unused otherwise)
    const float4 Cc = P->c;
    const v3 v1 = mk(B.z, B.w, Cc.x), v2 = mk(Cc.y, Cc.z, Cc.w);
    const v3 p = add(o, muls(d, tt));
    const v3 e1 = sub(v2, v1), e2 = sub(v0, v2);
    const float inv_area = 1.0f / dot(cross(e1, e2), n);
    const float uu = dot(cross(e1, sub(p, v1)), n) * inv_area;
    if (uu < 0 || uu > 1.0f) return false;
    const float vv = dot(cross(e2, sub(p, v2)), n) * inv_area;
    if (vv < 0 || (uu + vv) > 1.0f) return false;
    t = tt;
    u = uu;
    v = vv;
    return true;
}

}  // namespace rtgd
