/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of RTBase's render loop, used as the
 * parity checker (tests/, __graft_entry__.smoke()) and as the CPU baseline leg of bench.py.
 * The product (librtg.so / librth.so) never links or calls this file.
 *
 * It restates, function for function and in the reference's floating-point operation order:
 *   RayTracer::render / pathTracerTileBased / getTileID / renderTile  RTBase/Renderer.h:795-885
 *   RayTracer::pathTrace                                             RTBase/Renderer.h:328-392
 *   RayTracer::computeDirect                                         RTBase/Renderer.h:423-473
 *   RayTracer::computeDirectMIS (+ convertPDFAreaToSolidAngle, balanceHeuristic) Renderer.h:408-557
 *   RayTracer::adaptiveRender / adaptiveSampling / sampleTileWithWeight  RTBase/Renderer.h:583-749
 *   RayTracer::lightTracer / lightTrace_init / lightTracePath / connectToCamera  Renderer.h:221-326
 *   Camera::projectOntoCamera                                         RTBase/Scene.h:55-69
 *   RayTracer::instantRadiosity / traceVPLs / VPLTracePath / computeVPLsContribution  Renderer.h:82-218
 *   Scene::traverse / visible / sampleLight / calculateShadingData   RTBase/Scene.h:107-203
 *   BVHNode::traverse / traverseVisible (left-first DFS, no culling) RTBase/Geometry.h:399-462
 *   AABB::rayAABB, Triangle::init / rayIntersect / sample / gNormal  RTBase/Geometry.h:72-184
 *   Camera::generateRay                                              RTBase/Scene.h:43-54
 *   Diffuse/Mirror/Glass BSDF + the Lambert stubs                    RTBase/Materials.h:118-465
 *   AreaLight / EnvironmentMap sample + evaluate                     RTBase/Lights.h:30-201
 *   Texture::sample                                                  RTBase/Imaging.h:72-94
 *   SamplingDistributions, SphericalCoordinates, Frame               RTBase/Sampling.h, Core.h
 * on the flattened Scene of include/rtg.h (the host front-end's output), with the deterministic
 * PCG32 sampler of SURVEY.md Appendix B injected in place of MTRandom (Sampling.h:13-26).
 *
 * Argument-evaluation order: the reference writes cosineSampleHemisphere(sampler.next(),
 * sampler.next()) (Materials.h:129) and uniformSampleSphere(sampler.next(), sampler.next())
 * (Lights.h:145); g++ evaluates those arguments right to left, so the FIRST draw becomes r2.
 *
 * Transcendentals: built twice. ORACLE_LIBM=1 calls the C library's acosf/sinf/cosf/atan2f
 * (what the reference gets on Linux); otherwise the shared bit-reproducible rtm_* functions of
 * include/rtg_math.h (what the GPU build uses), so GPU-vs-oracle can be compared bit for bit.
 * Compile with -ffp-contract=off.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rtg.h"
#include "../include/rtg_math.h"

#if ORACLE_LIBM
#define O_ACOSF acosf
#define O_SINF sinf
#define O_COSF cosf
#define O_ATAN2F atan2f
#else
#define O_ACOSF rtm_acosf
#define O_SINF rtm_sinf
#define O_COSF rtm_cosf
#define O_ATAN2F rtm_atan2f
#endif

#define O_EPS 1e-4f
#define O_PI 3.14159265358979323846 /* M_PI */

typedef struct { float x, y, z, w; } V3; /* Core.h Vec3: 16 B, constructors set w = 1 */
typedef struct { float r, g, b; } Col;

static V3 v3(float x, float y, float z) { V3 v; v.x = x; v.y = y; v.z = z; v.w = 1.0f; return v; }
static V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static V3 vmuls(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static V3 vmulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static float vdot(V3 a, V3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
static V3 vcross(V3 a, V3 b) { return v3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)); }
static float vlen2(V3 a) { return ((a.x * a.x) + (a.y * a.y)) + (a.z * a.z); }
static float vlen(V3 a) { return sqrtf(((a.x * a.x) + (a.y * a.y)) + (a.z * a.z)); }
static V3 vnorm(V3 a) { float l = 1.0f / sqrtf(((a.x * a.x) + (a.y * a.y)) + (a.z * a.z)); return v3(a.x * l, a.y * l, a.z * l); }
static V3 Vmin(V3 a, V3 b) { return v3(a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z); }
static V3 Vmax(V3 a, V3 b) { return v3(a.x > b.x ? a.x : b.x, a.y > b.y ? a.y : b.y, a.z > b.z ? a.z : b.z); }
static float std_max(float a, float b) { return (a < b) ? b : a; }
static float std_min(float a, float b) { return (b < a) ? b : a; }
static float win_max(float a, float b) { return a > b ? a : b; } /* windows.h macro */
static float win_min(float a, float b) { return a < b ? a : b; }

static Col col(float r, float g, float b) { Col c; c.r = r; c.g = g; c.b = b; return c; }
static Col cadd(Col a, Col b) { return col(a.r + b.r, a.g + b.g, a.b + b.b); }
static Col cmul(Col a, Col b) { return col(a.r * b.r, a.g * b.g, a.b * b.b); }
static Col cmuls(Col a, float s) { return col(a.r * s, a.g * s, a.b * s); }
static Col cdivs(Col a, float s) { return col(a.r / s, a.g / s, a.b / s); }
static float clum(Col c) { return ((0.2126f * c.r) + (0.7152f * c.g)) + (0.0722f * c.b); }

typedef struct { V3 u, v, w; } Frame;
static Frame frame_from(V3 n) { /* Core.h:513-527 */
    Frame f;
    f.w = vnorm(n);
    if (fabsf(f.w.x) > fabsf(f.w.y)) {
        float l = 1.0f / sqrtf(f.w.x * f.w.x + f.w.z * f.w.z);
        f.u = v3(f.w.z * l, 0.0f, -f.w.x * l);
    } else {
        float l = 1.0f / sqrtf(f.w.y * f.w.y + f.w.z * f.w.z);
        f.u = v3(0, f.w.z * l, -f.w.y * l);
    }
    f.v = vcross(f.w, f.u);
    return f;
}
static V3 to_local(const Frame* f, V3 a) { return v3(vdot(a, f->u), vdot(a, f->v), vdot(a, f->w)); }
static V3 to_world(const Frame* f, V3 a) { return vadd(vadd(vmuls(f->u, a.x), vmuls(f->v, a.y)), vmuls(f->w, a.z)); }

/* ------------------------------------------------------------------ sampler */
typedef struct { uint64_t s, inc; } Pcg;
static uint32_t pcg_u32(Pcg* p) {
    uint64_t o = p->s;
    p->s = o * 6364136223846793005ULL + p->inc;
    uint32_t x = (uint32_t)(((o >> 18u) ^ o) >> 27u);
    uint32_t r = (uint32_t)(o >> 59u);
    return (x >> r) | (x << ((0u - r) & 31u));
}
static void pcg_init(Pcg* p, uint64_t seed, uint64_t seq) {
    p->s = 0;
    p->inc = (seq << 1u) | 1u;
    pcg_u32(p);
    p->s += seed;
    pcg_u32(p);
}
static float pcg_next(Pcg* p) { return (float)(pcg_u32(p) >> 8) * (1.0f / 16777216.0f); }

/* ------------------------------------------------------------------ scene */
/* Scene records in the reference's memory layout, so that the tile renderer's cache behaviour (and
 * so the CPU baseline of bench.py) is the reference's: Vec3 is 16 B (Core.h), Vertex 40 B, Triangle
 * 180 B in one std::vector (Geometry.h:62-71), BVHNode 56 B allocated one by one with `new`
 * (64-B stride: 8-B allocator header), children in pairs l, r and then l's subtree before r's
 * (BVHNode::buildRecursive, Geometry.h:387-390). The arithmetic does not depend on the layout. */
typedef struct { V3 p; V3 n; float u, v; } Vtx;
typedef struct {
    Vtx vx[3];
    V3 e1, e2, nrm;
    float area, d;
    uint32_t mat;
} Tri;
typedef struct { V3 mn, mx; int r, r_hi, l, l_hi; int start, end; int heap[2]; } Node;
_Static_assert(sizeof(Tri) == 180, "reference Triangle is 180 B");
_Static_assert(sizeof(Node) == 64, "reference BVHNode allocation stride is 64 B");
typedef struct { int w, h; const float* t; } Tex;

struct or_scene {
    int ntri, nnode, nlight, env_tex, max_depth, integrator;
    Tri* tri;
    Node* node;
    rtg_material* mat;
    Tex* tex;
    float* texels;
    int* light;
    rtg_camera cam;
    rtg_camera_proj proj;
    int W, H;
};

typedef struct {
    uint64_t ext_rays, shadow_rays, nodes, tris;
} Counts;

/* Optional per-path event log (or_path_events): the first differing event of two builds' paths
 * names where a divergent pixel's paths part ways. Thread-local, off unless set. */
typedef struct { float* ev; int n, cap; } EvLog;
static __thread EvLog* g_ev;
static void ev_push(float kind, float a, float b, float c, float d) {
    if (!g_ev) return;
    if (g_ev->n < g_ev->cap) {
        float* e = g_ev->ev + (size_t)g_ev->n * 5;
        e[0] = kind; e[1] = a; e[2] = b; e[3] = c; e[4] = d;
    }
    g_ev->n++;
}

typedef struct { V3 o, dir, inv; } Ray;
static Ray ray_make(V3 o, V3 d) { Ray r; r.o = o; r.dir = d; r.inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); return r; }

/* AABB::rayAABB (Geometry.h:173-184) */
static int ray_aabb(const Node* b, const Ray* r) {
    V3 tmin = vmulv(vsub(b->mn, r->o), r->inv);
    V3 tmax = vmulv(vsub(b->mx, r->o), r->inv);
    V3 ten = Vmin(tmin, tmax), tex = Vmax(tmin, tmax);
    float te = std_max(std_max(ten.x, ten.y), ten.z);
    float tx = std_min(std_min(tex.x, tex.y), tex.z);
    if (tx < te || tx < 0) return 0;
    return 1;
}

/* Triangle::rayIntersect (Geometry.h:89-105) */
static int tri_hit(const Tri* T, const Ray* r, float* t, float* u, float* v) {
    float denom = vdot(T->nrm, r->dir);
    if (denom == 0) return 0;
    *t = (T->d - vdot(T->nrm, r->o)) / denom;
    if (*t < 0) return 0;
    V3 p = vadd(r->o, vmuls(r->dir, *t));
    float inv_area = 1.0f / vdot(vcross(T->e1, T->e2), T->nrm);
    *u = vdot(vcross(T->e1, vsub(p, T->vx[1].p)), T->nrm) * inv_area;
    if (*u < 0 || *u > 1.0f) return 0;
    *v = vdot(vcross(T->e2, vsub(p, T->vx[2].p)), T->nrm) * inv_area;
    if (*v < 0 || (*u + *v) > 1.0f) return 0;
    return 1;
}

typedef struct { int id; float t, alpha, beta, gamma; } Isect;

/* BVHNode::traverse (Geometry.h:399-427): recursive left-then-right, no ordering/culling */
static void traverse(const struct or_scene* s, int ni, const Ray* r, Isect* is, Counts* c) {
    const Node* n = &s->node[ni];
    if (c) c->nodes++;
    if (!ray_aabb(n, r)) return;
    if (n->l < 0 && n->r < 0) {
        for (int i = n->start; i < n->end; i++) {
            float t, u, v;
            if (c) c->tris++;
            if (tri_hit(&s->tri[i], r, &t, &u, &v)) {
                if (t < is->t && t > O_EPS) {
                    is->t = t;
                    is->id = i;
                    is->alpha = u;
                    is->beta = v;
                    is->gamma = 1.0f - (u + v);
                }
            }
        }
        return;
    }
    if (n->l >= 0) traverse(s, n->l, r, is, c);
    if (n->r >= 0) traverse(s, n->r, r, is, c);
}

/* BVHNode::traverseVisible (Geometry.h:435-462) */
static int traverse_visible(const struct or_scene* s, int ni, const Ray* r, float maxT, Counts* c) {
    const Node* n = &s->node[ni];
    if (c) c->nodes++;
    if (!ray_aabb(n, r)) return 1;
    if (n->l < 0 && n->r < 0) {
        for (int i = n->start; i < n->end; i++) {
            float t, u, v;
            if (c) c->tris++;
            if (tri_hit(&s->tri[i], r, &t, &u, &v)) {
                if (t >= maxT || t <= O_EPS) continue;
                return 0;
            }
        }
        return 1;
    }
    if (!traverse_visible(s, n->l, r, maxT, c)) return 0;
    return traverse_visible(s, n->r, r, maxT, c);
}

static Isect scene_traverse(const struct or_scene* s, const Ray* r, Counts* c) {
    Isect is;
    is.id = -1;
    is.t = FLT_MAX;
    is.alpha = is.beta = is.gamma = 0;
    if (c) c->ext_rays++;
    traverse(s, 0, r, &is, c);
    ev_push(1, (float)is.id, is.t, is.alpha, is.beta); /* closest hit (id -1: miss) */
    return is;
}

/* Scene::visible (Scene.h:161-169) */
static int scene_visible(const struct or_scene* s, V3 p1, V3 p2, Counts* c) {
    V3 dir = vsub(p2, p1);
    float maxT = vlen(dir) - (2.0f * O_EPS);
    dir = vnorm(dir);
    Ray r = ray_make(vadd(p1, vmuls(dir, O_EPS)), dir);
    if (c) c->shadow_rays++;
    int vis = traverse_visible(s, 0, &r, maxT, c);
    ev_push(3, (float)vis, maxT, 0, 0); /* shadow ray */
    return vis;
}

/* Texture::sample (Imaging.h:72-94) */
static Col tex_sample(const struct or_scene* s, int ti, float tu, float tv) {
    const Tex* T = &s->tex[ti];
    float u = std_max(0.0f, fabsf(tu)) * T->w;
    float v = std_max(0.0f, fabsf(tv)) * T->h;
    int x = (int)floorf(u), y = (int)floorf(v);
    float fu = u - x, fv = v - y;
    float w0 = (1.0f - fu) * (1.0f - fv), w1 = fu * (1.0f - fv), w2 = (1.0f - fu) * fv, w3 = fu * fv;
    x = x % T->w;
    y = y % T->h;
    const float* a = T->t + (size_t)(y * T->w + x) * 3;
    const float* b = T->t + (size_t)(y * T->w + ((x + 1) % T->w)) * 3;
    const float* cc = T->t + (size_t)(((y + 1) % T->h) * T->w + x) * 3;
    const float* d = T->t + (size_t)(((y + 1) % T->h) * T->w + ((x + 1) % T->w)) * 3;
    Col s0 = col(a[0], a[1], a[2]), s1 = col(b[0], b[1], b[2]), s2 = col(cc[0], cc[1], cc[2]), s3 = col(d[0], d[1], d[2]);
    return cadd(cadd(cadd(cmuls(s0, w0), cmuls(s1, w1)), cmuls(s2, w2)), cmuls(s3, w3));
}

/* SamplingDistributions (Sampling.h:44-69) + SphericalCoordinates (Core.h:547-550) */
static V3 sph_to_world(float theta, float phi) {
    return v3(O_COSF(phi) * O_SINF(theta), O_SINF(phi) * O_SINF(theta), O_COSF(theta));
}
static V3 cosine_sample_hemisphere(float r1, float r2) {
    float theta = O_ACOSF(sqrtf(r1));
    float phi = (float)(2.0f * O_PI * r2);
    return sph_to_world(theta, phi);
}
static V3 uniform_sample_sphere(float r1, float r2) {
    float theta = O_ACOSF(1 - 2 * r1);
    float phi = (float)(2.0f * O_PI * r2);
    return sph_to_world(theta, phi);
}

/* EnvironmentMap::evaluate (Lights.h:150-157) */
static Col env_eval(const struct or_scene* s, V3 wi) {
    float u = O_ATAN2F(wi.z, wi.x);
    u = (float)((u < 0.0f) ? u + (2.0f * O_PI) : u);
    u = (float)(u / (2.0f * O_PI));
    float v = (float)(O_ACOSF(wi.y) / O_PI);
    return tex_sample(s, s->env_tex, u, v);
}

/* fresnelDielectric (Materials.h:55-77) */
static float fresnel_dielectric(float cos_i, float ior_int, float ior_ext, V3* wt, V3 wol) {
    float ior = ior_int / ior_ext;
    float sin_i = sqrtf(1 - (cos_i * cos_i));
    float sin_t = ior * sin_i;
    float ior2sin2 = (ior * ior) * (1 - (cos_i * cos_i));
    if (ior2sin2 > 1.0f) return 1.0f;
    float cos_t = sqrtf(1 - (sin_t * sin_t));
    *wt = v3(-ior * wol.x, -ior * wol.y, -cos_t);
    float fpa = (cos_i - ior * cos_t) / (cos_i + ior * cos_t);
    float fpe = (ior * cos_i - cos_t) / (ior * cos_i + ior * cos_t);
    float avg = ((fpa * fpa) + (fpe * fpe)) * 0.5f;
    return std_max(0.0f, std_min(1.0f, avg));
}

typedef struct {
    V3 x, wo, sN;
    float tu, tv;
    Frame frame;
    const rtg_material* bsdf;
    float t;
} Shading;

/* Scene::calculateShadingData (Scene.h:174-203) */
static Shading shading_data(const struct or_scene* s, const Isect* is, const Ray* r) {
    Shading sd;
    memset(&sd, 0, sizeof(sd));
    sd.t = is->t;
    sd.wo = vneg(r->dir);
    if (!(is->t < FLT_MAX)) return sd;
    const Tri* T = &s->tri[is->id];
    sd.x = vadd(r->o, vmuls(r->dir, is->t));
    V3 n = vadd(vadd(vmuls(T->vx[0].n, is->alpha), vmuls(T->vx[1].n, is->beta)), vmuls(T->vx[2].n, is->gamma));
    sd.sN = vnorm(n);
    sd.tu = (T->vx[0].u * is->alpha + T->vx[1].u * is->beta) + T->vx[2].u * is->gamma;
    sd.tv = (T->vx[0].v * is->alpha + T->vx[1].v * is->beta) + T->vx[2].v * is->gamma;
    sd.bsdf = &s->mat[T->mat];
    if (sd.bsdf->two_sided && vdot(sd.wo, sd.sN) < 0) sd.sN = vneg(sd.sN);
    sd.frame = frame_from(sd.sN);
    return sd;
}

static int is_spec(const rtg_material* m) { return m->kind == RTG_MAT_MIRROR || m->kind == RTG_MAT_GLASS; }
static int is_light(const rtg_material* m) { return clum(col(m->emission[0], m->emission[1], m->emission[2])) > 0; }

/* BSDF::evaluate for the non-specular kinds (albedo / M_PI as float) */
static Col bsdf_eval(const struct or_scene* s, const Shading* sd) {
    return cdivs(tex_sample(s, sd->bsdf->texture, sd->tu, sd->tv), (float)O_PI);
}

/* RayTracer::computeDirect (Renderer.h:423-473) */
static Col compute_direct(const struct or_scene* s, const Shading* sd, Pcg* smp, Counts* c) {
    if (is_spec(sd->bsdf)) return col(0.0f, 0.0f, 0.0f);
    float pmf = 1.f / (float)s->nlight;
    int li = (int)((float)s->nlight * pcg_next(smp));
    if (s->nlight - 1 < li) li = s->nlight - 1; /* (std::min)(a, b) */
    int lt = s->light[li];
    if (lt >= 0) { /* AreaLight::sample -> Triangle::sample (Geometry.h:114-126) */
        const Tri* T = &s->tri[lt];
        float r1 = pcg_next(smp);
        float r2 = pcg_next(smp);
        float alpha = 1 - sqrtf(r1);
        float beta = r2 * sqrtf(r1);
        float gamma = 1.0f - (alpha + beta);
        float pdf = 1.0f / T->area;
        V3 p = vadd(vadd(vmuls(T->vx[0].p, alpha), vmuls(T->vx[1].p, beta)), vmuls(T->vx[2].p, gamma));
        ev_push(2, (float)li, p.x, p.y, p.z); /* area light sample point */
        const float* e = s->mat[T->mat].emission;
        Col emitted = col(e[0], e[1], e[2]);
        V3 wi = vsub(p, sd->x);
        float l = vlen2(wi);
        wi = vnorm(wi);
        V3 gn = vmuls(T->nrm, vdot(T->vx[0].n, T->nrm) > 0 ? 1.0f : -1.0f); /* Triangle::gNormal */
        float G = (win_max(vdot(wi, sd->sN), 0.0f) * win_max(-vdot(wi, gn), 0.0f)) / l;
        if (G > 0) {
            if (scene_visible(s, sd->x, p, c))
                return cdivs(cmuls(cmul(bsdf_eval(s, sd), emitted), G), pmf * pdf);
        }
    } else { /* EnvironmentMap::sample */
        float q2 = pcg_next(smp);
        float q1 = pcg_next(smp);
        V3 wi = uniform_sample_sphere(q1, q2);
        ev_push(2, (float)li, wi.x, wi.y, wi.z); /* environment sample direction */
        float pdf = (float)(1.0f / (4.0f * O_PI));
        Col emitted = env_eval(s, wi);
        float G = win_max(vdot(wi, sd->sN), 0.0f);
        if (G > 0) {
            if (scene_visible(s, sd->x, vadd(sd->x, vmuls(wi, 10000.0f)), c))
                return cdivs(cmuls(cmul(bsdf_eval(s, sd), emitted), G), pmf * pdf);
        }
    }
    return col(0.0f, 0.0f, 0.0f);
}

/* BSDF::PDF of the non-specular kinds: cosineHemispherePDF(frame.toLocal(wi)) (Materials.h:136-140) */
static float bsdf_pdf(const Shading* sd, V3 wi) {
    V3 wl = to_local(&sd->frame, wi);
    return (float)((wl.z >= 0.0f) ? (wl.z / O_PI) : 0.0f);
}
/* convertPDFAreaToSolidAngle / balanceHeuristic (Renderer.h:408-422) */
static float area_to_solid(float pdf_area, float dist2, float cos_theta) {
    if (cos_theta > 0.0f) return pdf_area * dist2 / cos_theta;
    return 0.0f;
}
static float balance(float pa, float pb) { return pa / (pa + pb); }

/* BSDF::sample for the three effective behaviours */
static V3 bsdf_sample(const struct or_scene* s, const Shading* sd, Pcg* smp, Col* refl, float* pdf) {
    const rtg_material* m = sd->bsdf;
    Col alb = tex_sample(s, m->texture, sd->tu, sd->tv);
    if (m->kind == RTG_MAT_DIFFUSE || m->kind == RTG_MAT_LAMBERT) {
        float q2 = pcg_next(smp); /* cosineSampleHemisphere(sampler.next(), sampler.next()) */
        float q1 = pcg_next(smp);
        V3 wl = cosine_sample_hemisphere(q1, q2);
        if (m->kind == RTG_MAT_DIFFUSE) *pdf = (float)((wl.z >= 0.0f) ? (wl.z / O_PI) : 0.0f); /* cosineHemispherePDF */
        else *pdf = (float)(wl.z / O_PI);                                                      /* Lambert stubs */
        *refl = cdivs(alb, (float)O_PI);
        return to_world(&sd->frame, wl);
    }
    if (m->kind == RTG_MAT_MIRROR) { /* Materials.h:167-177 */
        V3 wol = to_local(&sd->frame, sd->wo);
        *pdf = 1.0f;
        *refl = alb;
        return to_world(&sd->frame, v3(-wol.x, -wol.y, wol.z));
    }
    /* GlassBSDF::sample (Materials.h:265-294) */
    V3 wol = to_local(&sd->frame, sd->wo);
    float cos_i = fabsf(wol.z);
    int enter = wol.z > 0.0f;
    float eta_i = enter ? m->ext_ior : m->int_ior;
    float eta_t = enter ? m->int_ior : m->ext_ior;
    V3 wt = v3(0, 0, 0), wi;
    float R = fresnel_dielectric(cos_i, eta_i, eta_t, &wt, wol);
    if (!enter) wt.z = -wt.z;
    int reflect = (R == 1.0f || pcg_next(smp) < R);
    if (reflect) {
        wi = v3(-wol.x, -wol.y, wol.z);
        *pdf = R;
        *refl = cmuls(alb, R);
    } else {
        wi = wt;
        *pdf = 1.0f - R;
        *refl = cmuls(alb, 1.0f - R);
    }
    return to_world(&sd->frame, wi);
}

/* RayTracer::computeDirectMIS (Renderer.h:474-557) */
static Col compute_direct_mis(const struct or_scene* s, const Shading* sd, Pcg* smp, Counts* c) {
    if (is_spec(sd->bsdf)) return col(0.0f, 0.0f, 0.0f);
    Col result = col(0.0f, 0.0f, 0.0f);
    float pmf = 1.f / (float)s->nlight;
    int li = (int)((float)s->nlight * pcg_next(smp));
    if (s->nlight - 1 < li) li = s->nlight - 1;
    int lt = s->light[li];
    float pdf;
    if (lt >= 0) {
        const Tri* T = &s->tri[lt];
        float r1 = pcg_next(smp);
        float r2 = pcg_next(smp);
        float alpha = 1 - sqrtf(r1);
        float beta = r2 * sqrtf(r1);
        float gamma = 1.0f - (alpha + beta);
        pdf = 1.0f / T->area;
        V3 p = vadd(vadd(vmuls(T->vx[0].p, alpha), vmuls(T->vx[1].p, beta)), vmuls(T->vx[2].p, gamma));
        ev_push(2, (float)li, p.x, p.y, p.z); /* area light sample point */
        const float* e = s->mat[T->mat].emission;
        Col emitted = col(e[0], e[1], e[2]);
        V3 wi = vsub(p, sd->x);
        float l = vlen2(wi);
        wi = vnorm(wi);
        V3 gn = vmuls(T->nrm, vdot(T->vx[0].n, T->nrm) > 0 ? 1.0f : -1.0f);
        float cos_surface = win_max(vdot(wi, sd->sN), 0.0f);
        float cos_light = win_max(-vdot(wi, gn), 0.0f);
        float G = cos_surface * cos_light / l;
        if (G > 0) {
            if (scene_visible(s, sd->x, p, c)) {
                float pdf_bsdf = bsdf_pdf(sd, wi);
                float pdf_light = area_to_solid(pdf * pmf, l, cos_light);
                float w = balance(pdf_light, pdf_bsdf);
                result = cadd(result, cdivs(cmuls(cmuls(cmul(bsdf_eval(s, sd), emitted), G), w), pmf * pdf));
            }
        }
    } else {
        float q2 = pcg_next(smp);
        float q1 = pcg_next(smp);
        V3 wi = uniform_sample_sphere(q1, q2);
        pdf = (float)(1.0f / (4.0f * O_PI));
        Col emitted = env_eval(s, wi);
        float G = win_max(vdot(wi, sd->sN), 0.0f);
        if (G > 0) {
            if (scene_visible(s, sd->x, vadd(sd->x, vmuls(wi, 10000.0f)), c))
                return cdivs(cmuls(cmul(bsdf_eval(s, sd), emitted), G), pmf * pdf);
        }
    }
    Col val;
    float pdf_b;
    V3 wib = bsdf_sample(s, sd, smp, &val, &pdf_b);
    Ray r = ray_make(vadd(sd->x, vmuls(wib, O_EPS)), wib);
    Isect is = scene_traverse(s, &r, c);
    Shading sl = shading_data(s, &is, &r);
    if (sl.t < FLT_MAX) {
        if (is_light(sl.bsdf)) {
            const float* e = sl.bsdf->emission;
            Col emitted2 = col(e[0], e[1], e[2]);
            V3 wi = vsub(sl.x, sd->x);
            float dist2 = vlen2(wi);
            wi = vnorm(wi);
            float cos_light = win_max(0.0f, vdot(vneg(wi), sl.sN));
            float pdf_light = area_to_solid(pdf * pmf, dist2, cos_light);
            float w = balance(pdf_b, pdf_light);
            result = cadd(result, cdivs(cmuls(cmuls(cmul(val, emitted2), win_max(0.0f, vdot(wib, sd->sN))), w), pdf_b));
        }
    }
    return result;
}

/* RayTracer::pathTrace (Renderer.h:328-392) */
static Col path_trace(const struct or_scene* s, Ray* r, Col* thr, int depth, Pcg* smp, int can_hit, Counts* c) {
    Isect is = scene_traverse(s, r, c);
    Shading sd = shading_data(s, &is, r);
    if (sd.t < FLT_MAX) {
        if (is_light(sd.bsdf)) {
            if (can_hit) {
                const float* e = sd.bsdf->emission;
                return cmul(*thr, col(e[0], e[1], e[2]));
            }
            return col(0.0f, 0.0f, 0.0f);
        }
        Col direct = cmul(*thr, compute_direct(s, &sd, smp, c));
        if (depth > s->max_depth) return direct;
        float rrp = win_min(clum(*thr), 0.9f);
        float q = pcg_next(smp);
        ev_push(4, q, rrp, (float)depth, 0); /* Russian roulette */
        if (q < rrp) *thr = cdivs(*thr, rrp);
        else return direct;
        Col ind;
        float pdf;
        V3 wi = bsdf_sample(s, &sd, smp, &ind, &pdf);
        ev_push(5, wi.x, wi.y, wi.z, pdf); /* BSDF sample */
        if (is_spec(sd.bsdf)) *thr = cdivs(cmul(*thr, ind), pdf);
        else *thr = cdivs(cmuls(cmul(*thr, ind), fabsf(vdot(wi, sd.sN))), pdf);
        *r = ray_make(vadd(sd.x, vmuls(wi, O_EPS)), wi);
        return cadd(direct, path_trace(s, r, thr, depth + 1, smp, is_spec(sd.bsdf), c));
    }
    if (s->env_tex < 0) return col(0.0f, 0.0f, 0.0f); /* BackgroundColour(0,0,0) */
    return env_eval(s, r->dir);
}

/* Camera::generateRay (Scene.h:43-54) */
static Ray camera_ray(const struct or_scene* s, float x, float y) {
    const rtg_camera* c = &s->cam;
    float xp = x / c->width;
    float yp = 1.0f - (y / c->height);
    xp = (xp * 2.0f) - 1.0f;
    yp = (yp * 2.0f) - 1.0f;
    const float* m = c->inv_proj;
    V3 d = v3(((xp * m[0] + yp * m[1]) + 1.0f * m[2]) + m[3], ((xp * m[4] + yp * m[5]) + 1.0f * m[6]) + m[7],
              ((xp * m[8] + yp * m[9]) + 1.0f * m[10]) + m[11]);
    const float* k = c->camera;
    d = v3((d.x * k[0] + d.y * k[1]) + d.z * k[2], (d.x * k[4] + d.y * k[5]) + d.z * k[6], (d.x * k[8] + d.y * k[9]) + d.z * k[10]);
    d = vnorm(d);
    return ray_make(v3(c->origin[0], c->origin[1], c->origin[2]), d);
}

/* RayTracer::direct (Renderer.h:393-407): emission or one NEE sample at the first hit; 0 on a miss */
static Col direct_only(const struct or_scene* s, Ray* r, Pcg* smp, Counts* c) {
    Isect is = scene_traverse(s, r, c);
    Shading sd = shading_data(s, &is, r);
    if (sd.t < FLT_MAX) {
        if (is_light(sd.bsdf)) return col(sd.bsdf->emission[0], sd.bsdf->emission[1], sd.bsdf->emission[2]);
        return compute_direct(s, &sd, smp, c);
    }
    return col(0.0f, 0.0f, 0.0f);
}

/* RayTracer::direct with computeDirectMIS in place of computeDirect */
static Col direct_mis_only(const struct or_scene* s, Ray* r, Pcg* smp, Counts* c) {
    Isect is = scene_traverse(s, r, c);
    Shading sd = shading_data(s, &is, r);
    if (sd.t < FLT_MAX) {
        if (is_light(sd.bsdf)) return col(sd.bsdf->emission[0], sd.bsdf->emission[1], sd.bsdf->emission[2]);
        return compute_direct_mis(s, &sd, smp, c);
    }
    return col(0.0f, 0.0f, 0.0f);
}

/* RayTracer::albedo (Renderer.h:558-571): emission, BSDF::evaluate(sd, (0,1,0)) or background */
static Col albedo_only(const struct or_scene* s, Ray* r, Counts* c) {
    Isect is = scene_traverse(s, r, c);
    Shading sd = shading_data(s, &is, r);
    if (sd.t < FLT_MAX) {
        const rtg_material* m = sd.bsdf;
        if (is_light(m)) return col(m->emission[0], m->emission[1], m->emission[2]);
        if (m->kind == RTG_MAT_MIRROR) return tex_sample(s, m->texture, sd.tu, sd.tv); /* Materials.h:178-183 */
        if (m->kind == RTG_MAT_GLASS) return col(0.0f, 0.0f, 0.0f);
        return bsdf_eval(s, &sd);
    }
    if (s->env_tex < 0) return col(0.0f, 0.0f, 0.0f);
    return env_eval(s, r->dir);
}

/* RayTracer::viewNormals (Renderer.h:572-582): |shading normal| at the first hit */
static Col normals_only(const struct or_scene* s, Ray* r, Counts* c) {
    Isect is = scene_traverse(s, r, c);
    if (is.t < FLT_MAX) {
        Shading sd = shading_data(s, &is, r);
        return col(fabsf(sd.sN.x), fabsf(sd.sN.y), fabsf(sd.sN.z));
    }
    return col(0.0f, 0.0f, 0.0f);
}

static Col pixel_sample(const struct or_scene* s, uint32_t pixel, uint32_t sample, uint64_t seed, Counts* c) {
    uint32_t x = pixel % (uint32_t)s->W, y = pixel / (uint32_t)s->W;
    Pcg smp;
    pcg_init(&smp, seed, ((uint64_t)pixel << 16) | sample);
    Ray r = camera_ray(s, x + 0.5f, y + 0.5f);
    Col thr = col(1.0f, 1.0f, 1.0f);
    switch (s->integrator) {
    case RTG_INTEGRATOR_DIRECT: return direct_only(s, &r, &smp, c);
    case RTG_INTEGRATOR_ALBEDO: return albedo_only(s, &r, c);
    case RTG_INTEGRATOR_NORMALS: return normals_only(s, &r, c);
    case RTG_INTEGRATOR_DIRECT_MIS: return direct_mis_only(s, &r, &smp, c);
    default: return path_trace(s, &r, &thr, 0, &smp, 1, c);
    }
}

/* ------------------------------------------------------------------ public C API (ctypes) */
typedef struct or_scene or_scene;

or_scene* or_create(const rtg_scene_desc* d, int max_depth) {
    if (!d || d->n_nodes == 0) return NULL;
    or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
    s->ntri = (int)d->n_tris;
    s->nnode = (int)d->n_nodes;
    s->nlight = (int)d->n_lights;
    s->env_tex = d->env_texture;
    s->max_depth = max_depth;
    s->cam = d->camera;
    s->proj = d->projection;
    s->W = (int)d->camera.width;
    s->H = (int)d->camera.height;
    s->tri = (Tri*)calloc((size_t)s->ntri + 1, sizeof(Tri));
    for (int i = 0; i < s->ntri; ++i) { /* Triangle::init (Geometry.h:72-83) */
        Tri* T = &s->tri[i];
        for (int k = 0; k < 3; ++k) {
            const float* p = d->positions + (size_t)i * 9 + k * 3;
            const float* n = d->normals + (size_t)i * 9 + k * 3;
            T->vx[k].p = v3(p[0], p[1], p[2]);
            T->vx[k].n = v3(n[0], n[1], n[2]);
            T->vx[k].u = d->uvs[(size_t)i * 6 + k * 2];
            T->vx[k].v = d->uvs[(size_t)i * 6 + k * 2 + 1];
        }
        T->mat = d->material[i];
        T->e1 = vsub(T->vx[2].p, T->vx[1].p);
        T->e2 = vsub(T->vx[0].p, T->vx[2].p);
        T->nrm = vnorm(vcross(T->e1, T->e2));
        T->area = vlen(vcross(T->e1, T->e2)) * 0.5f;
        T->d = vdot(T->nrm, T->vx[0].p);
    }
    /* node order of the reference's allocations: root, then for every internal node its (l, r) pair
     * followed by l's subtree and r's subtree (an explicit stack of pending r subtrees) */
    s->node = (Node*)calloc((size_t)s->nnode, sizeof(Node));
    int* pos = (int*)malloc((size_t)s->nnode * sizeof(int));
    int* stk = (int*)malloc(((size_t)s->nnode + 1) * sizeof(int));
    int next = 0, top = 0;
    pos[0] = next++;
    stk[top++] = 0;
    while (top > 0) {
        int i = stk[--top];
        for (;;) {
            const int32_t* L = d->node_links + (size_t)i * 4;
            if (L[0] < 0 || L[1] < 0) break;
            pos[L[0]] = next++;
            pos[L[1]] = next++;
            stk[top++] = L[1];
            i = L[0];
        }
    }
    for (int i = 0; i < s->nnode; ++i) {
        const float* b = d->node_bounds + (size_t)i * 6;
        const int32_t* L = d->node_links + (size_t)i * 4;
        Node* n = &s->node[pos[i]];
        n->mn = v3(b[0], b[1], b[2]);
        n->mx = v3(b[3], b[4], b[5]);
        n->l = L[0] >= 0 ? pos[L[0]] : L[0];
        n->r = L[1] >= 0 ? pos[L[1]] : L[1];
        n->start = L[2];
        n->end = L[3];
    }
    free(pos);
    free(stk);
    s->mat = (rtg_material*)calloc((size_t)d->n_materials + 1, sizeof(rtg_material));
    memcpy(s->mat, d->materials, d->n_materials * sizeof(rtg_material));
    size_t total = 0;
    for (uint32_t i = 0; i < d->n_textures; ++i) total += (size_t)d->textures[i].width * d->textures[i].height * 3;
    s->texels = (float*)malloc((total + 1) * sizeof(float));
    s->tex = (Tex*)calloc((size_t)d->n_textures + 1, sizeof(Tex));
    size_t off = 0;
    for (uint32_t i = 0; i < d->n_textures; ++i) {
        size_t n = (size_t)d->textures[i].width * d->textures[i].height * 3;
        memcpy(s->texels + off, d->textures[i].texels, n * sizeof(float));
        s->tex[i].w = d->textures[i].width;
        s->tex[i].h = d->textures[i].height;
        s->tex[i].t = s->texels + off;
        off += n;
    }
    s->light = (int*)calloc((size_t)d->n_lights + 1, sizeof(int));
    memcpy(s->light, d->lights, d->n_lights * sizeof(int));
    return s;
}

void or_destroy(or_scene* s) {
    if (!s) return;
    free(s->tri); free(s->node); free(s->mat); free(s->tex); free(s->texels); free(s->light); free(s);
}

void or_set_max_depth(or_scene* s, int max_depth) { if (s) s->max_depth = max_depth; }
void or_set_integrator(or_scene* s, int integrator) { if (s) s->integrator = integrator; }

/* Per-path radiance for an explicit (pixel, sample) list: out n*3. */
int or_trace_paths(or_scene* s, const uint32_t* pixels, const uint32_t* samples, uint32_t n, uint64_t seed, float* out) {
    if (!s || s->nlight <= 0) return -1;
    for (uint32_t i = 0; i < n; ++i) {
        Col L = pixel_sample(s, pixels[i], samples[i], seed, NULL);
        out[i * 3] = L.r; out[i * 3 + 1] = L.g; out[i * 3 + 2] = L.b;
    }
    return 0;
}

/* Event log of one path (pixel, sample): up to cap events of 5 floats {kind, a, b, c, d}:
 * 1 closest hit {id, t, alpha, beta}, 2 light sample {index, point or direction}, 3 shadow ray
 * {visible, maxT}, 4 Russian roulette {draw, probability, depth}, 5 BSDF sample {wi, pdf}.
 * Returns the number of events (may exceed cap); radiance goes to L (3 floats). */
int or_path_events(or_scene* s, uint32_t pixel, uint32_t sample, uint64_t seed, float* ev, int cap, float* L) {
    if (!s || s->nlight <= 0) return -1;
    EvLog log = {ev, 0, cap};
    g_ev = &log;
    Col c = pixel_sample(s, pixel, sample, seed, NULL);
    g_ev = NULL;
    if (L) { L[0] = c.r; L[1] = c.g; L[2] = c.b; }
    return log.n;
}

/* RayTracer::render over tiles with a thread pool: for each sample (frame) in order, the
 * 32x32 tiles are pulled from a shared counter by `threads` workers (pathTracerTileBased /
 * getTileID), every pixel adds its path radiance to the film (renderTile + Film::splat).
 * film is W*H*3 and accumulated in place. counts (optional) receives
 * {paths, extension rays, shadow rays, node visits, triangle tests} when count != 0. */
typedef struct {
    or_scene* s;
    const uint32_t* tiles;
    uint32_t n_tiles;
    uint32_t sample;
    uint64_t seed;
    float* film;
    volatile uint32_t* next;
    int count;
    Counts cnt;
} Job;

static void render_tile(Job* j, uint32_t tile) {
    const int TS = 32;
    or_scene* s = j->s;
    uint32_t tx = (uint32_t)(s->W + TS - 1) / TS;
    uint32_t x0 = (tile % tx) * TS, y0 = (tile / tx) * TS;
    for (uint32_t y = y0; y < y0 + TS && y < (uint32_t)s->H; ++y)
        for (uint32_t x = x0; x < x0 + TS && x < (uint32_t)s->W; ++x) {
            uint32_t pix = y * (uint32_t)s->W + x;
            Col L = pixel_sample(s, pix, j->sample, j->seed, j->count ? &j->cnt : NULL);
            float* f = j->film + (size_t)pix * 3;
            f[0] = f[0] + L.r; f[1] = f[1] + L.g; f[2] = f[2] + L.b;
        }
}

static void* worker(void* arg) {
    Job* j = (Job*)arg;
    for (;;) {
        uint32_t k = __sync_fetch_and_add(j->next, 1u);
        if (k >= j->n_tiles) break;
        render_tile(j, j->tiles ? j->tiles[k] : k);
    }
    return NULL;
}

int or_render(or_scene* s, uint32_t first, uint32_t n_samples, uint64_t seed, const uint32_t* tiles, uint32_t n_tiles,
              int threads, float* film, uint64_t* counts, int count) {
    if (!s || !film || s->nlight <= 0) return -1;
    const int TS = 32;
    uint32_t ntiles_all = (uint32_t)((s->W + TS - 1) / TS) * (uint32_t)((s->H + TS - 1) / TS);
    uint32_t nt = tiles ? n_tiles : ntiles_all;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    Job jobs[256];
    pthread_t th[256];
    Counts total = {0, 0, 0, 0};
    for (uint32_t smp = first; smp < first + n_samples; ++smp) {
        volatile uint32_t next = 0;
        for (int t = 0; t < threads; ++t) {
            memset(&jobs[t], 0, sizeof(Job));
            jobs[t].s = s; jobs[t].tiles = tiles; jobs[t].n_tiles = nt; jobs[t].sample = smp;
            jobs[t].seed = seed; jobs[t].film = film; jobs[t].next = &next; jobs[t].count = count;
        }
        if (threads == 1) worker(&jobs[0]);
        else {
            for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
            for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
        }
        for (int t = 0; t < threads; ++t) {
            total.ext_rays += jobs[t].cnt.ext_rays; total.shadow_rays += jobs[t].cnt.shadow_rays;
            total.nodes += jobs[t].cnt.nodes; total.tris += jobs[t].cnt.tris;
        }
    }
    if (counts) {
        uint64_t npix = 0;
        for (uint32_t k = 0; k < nt; ++k) {
            uint32_t t = tiles ? tiles[k] : k;
            uint32_t tx = (uint32_t)(s->W + TS - 1) / TS;
            uint32_t x0 = (t % tx) * TS, y0 = (t / tx) * TS;
            uint32_t w = (uint32_t)s->W - x0 < (uint32_t)TS ? (uint32_t)s->W - x0 : (uint32_t)TS;
            uint32_t h = (uint32_t)s->H - y0 < (uint32_t)TS ? (uint32_t)s->H - y0 : (uint32_t)TS;
            npix += (uint64_t)w * h;
        }
        counts[0] = npix * n_samples;
        counts[1] = total.ext_rays; counts[2] = total.shadow_rays; counts[3] = total.nodes; counts[4] = total.tris;
    }
    return 0;
}

/* RayTracer::adaptiveRender (Renderer.h:583-749): adaptiveSampling per tile (init samples, variance
 * of the per-pixel means), weights = variance / total, sampleTileWithWeight (max((int)(sqrt(w) *
 * max_samples), min_samples) samples, film += their mean). Sample indices: pass 1 uses first ..
 * first+init-1, pass 2 first+init ... (the GPU build's convention for the deterministic sampler).
 * tile_samples (optional) receives the pass-2 counts. Single-threaded. */
int or_render_adaptive(or_scene* s, uint32_t first, uint64_t seed, uint32_t init, uint32_t max_samples,
                       uint32_t min_samples, float* film, uint32_t* tile_samples) {
    if (!s || !film || s->nlight <= 0 || init == 0) return -1;
    const int TS = 32;
    uint32_t tx = (uint32_t)(s->W + TS - 1) / TS, ty = (uint32_t)(s->H + TS - 1) / TS, nt = tx * ty;
    float* var = (float*)calloc(nt, sizeof(float));
    Col* est = (Col*)malloc(TS * TS * sizeof(Col));
    for (uint32_t t = 0; t < nt; ++t) {
        uint32_t x0 = (t % tx) * TS, y0 = (t / tx) * TS;
        int n = 0;
        for (uint32_t y = y0; y < y0 + TS && y < (uint32_t)s->H; ++y)
            for (uint32_t x = x0; x < x0 + TS && x < (uint32_t)s->W; ++x) {
                Col sum = col(0.0f, 0.0f, 0.0f);
                for (uint32_t i = 0; i < init; ++i) sum = cadd(sum, pixel_sample(s, y * (uint32_t)s->W + x, first + i, seed, NULL));
                est[n++] = cdivs(sum, (float)init);
            }
        Col gt = col(0.0f, 0.0f, 0.0f);
        for (int i = 0; i < n; ++i) gt = cadd(gt, est[i]);
        gt = cdivs(gt, (float)n);
        Col sq = col(0.0f, 0.0f, 0.0f);
        for (int i = 0; i < n; ++i) {
            Col d = col(est[i].r - gt.r, est[i].g - gt.g, est[i].b - gt.b);
            sq = cadd(sq, cmul(d, d));
        }
        var[t] = (((sq.r + sq.g) + sq.b) / 3.0f) / (float)(n - 1);
    }
    float total = 0.0f;
    for (uint32_t t = 0; t < nt; ++t) total += var[t];
    for (uint32_t t = 0; t < nt; ++t) {
        float w = (total > 0.0f) ? var[t] / total : 0.0f;
        w = sqrtf(w);
        int smp = (int)(w * (float)max_samples);
        smp = smp > (int)min_samples ? smp : (int)min_samples;
        if (tile_samples) tile_samples[t] = (uint32_t)smp;
        uint32_t x0 = (t % tx) * TS, y0 = (t / tx) * TS;
        for (uint32_t y = y0; y < y0 + TS && y < (uint32_t)s->H; ++y)
            for (uint32_t x = x0; x < x0 + TS && x < (uint32_t)s->W; ++x) {
                uint32_t pix = y * (uint32_t)s->W + x;
                Col c = col(0.0f, 0.0f, 0.0f);
                for (int i = 0; i < smp; ++i) c = cadd(c, pixel_sample(s, pix, first + init + (uint32_t)i, seed, NULL));
                c = cdivs(c, (float)smp);
                float* f = film + (size_t)pix * 3;
                f[0] = f[0] + c.r; f[1] = f[1] + c.g; f[2] = f[2] + c.b;
            }
    }
    free(var);
    free(est);
    return 0;
}

/* ------------------------------------------------------------------ light tracing (Renderer.h:221-326) */
/* Camera::projectOntoCamera (Scene.h:55-69) */
static int project_onto_camera(const struct or_scene* s, V3 p, float* x, float* y) {
    const float* m = s->proj.camera_to_view;
    V3 pv = v3(((p.x * m[0] + p.y * m[1]) + p.z * m[2]) + m[3], ((p.x * m[4] + p.y * m[5]) + p.z * m[6]) + m[7],
               ((p.x * m[8] + p.y * m[9]) + p.z * m[10]) + m[11]);
    const float* q = s->proj.proj;
    V3 v1 = v3(((pv.x * q[0] + pv.y * q[1]) + pv.z * q[2]) + q[3], ((pv.x * q[4] + pv.y * q[5]) + pv.z * q[6]) + q[7],
               ((pv.x * q[8] + pv.y * q[9]) + pv.z * q[10]) + q[11]);
    float w = (((q[12] * pv.x) + (q[13] * pv.y)) + (q[14] * pv.z)) + q[15];
    w = 1.0f / w;
    V3 pp = vmuls(v1, w);
    *x = (pp.x + 1.0f) * 0.5f;
    *y = (pp.y + 1.0f) * 0.5f;
    if (*x < 0 || *x > 1.0f || *y < 0 || *y > 1.0f) return 0;
    *x = *x * s->cam.width;
    *y = 1.0f - *y;
    *y = *y * s->cam.height;
    return 1;
}
/* (int)x with x86-64 cvttss2si semantics (NaN / out of range -> INT_MIN) */
static int trunc_x86(float x) { return (x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : (int)0x80000000; }
/* Film::splat, BoxFilter (size 0): film[(int)y * W + (int)x] += L * 1 / 1 (Imaging.h:209-232) */
static void splat(const struct or_scene* s, float* film, float x, float y, Col L) {
    int px = trunc_x86(x), py = trunc_x86(y);
    if (px >= 0 && (unsigned)px < (unsigned)s->W && py >= 0 && (unsigned)py < (unsigned)s->H) {
        float* f = film + ((size_t)py * (unsigned)s->W + (unsigned)px) * 3;
        f[0] = f[0] + ((L.r * 1.0f) / 1.0f);
        f[1] = f[1] + ((L.g * 1.0f) / 1.0f);
        f[2] = f[2] + ((L.b * 1.0f) / 1.0f);
    }
}
/* RayTracer::connectToCamera (Renderer.h:236-262) */
static void connect_to_camera(const struct or_scene* s, V3 p, V3 n, Col c, float* film, Counts* cnt) {
    float x, y;
    if (project_onto_camera(s, p, &x, &y)) {
        float A = s->proj.a_film;
        V3 org = v3(s->cam.origin[0], s->cam.origin[1], s->cam.origin[2]);
        V3 dir = vsub(org, p);
        float dist2 = vlen2(dir);
        dir = vnorm(dir);
        float cs = vdot(n, dir);
        float cc = vdot(v3(s->proj.view_direction[0], s->proj.view_direction[1], s->proj.view_direction[2]), vneg(dir));
        if (cs < 0.0f || cc < 0.0f) return;
        float G = (cs * cc) / dist2;
        if (!scene_visible(s, p, org, cnt)) return;
        float We = 1 / (A * ((cc * cc) * (cc * cc)));
        splat(s, film, x, y, cmuls(cmuls(c, We), G));
    }
}
/* AreaLight: samplePositionFromLight (Triangle::sample) + sampleDirectionFromLight (Lights.h:63-80) */
static void light_emit_sample(const struct or_scene* s, const Tri* T, Pcg* smp, V3* p, float* pdf_pos, V3* wi,
                              float* pdf_dir, V3* gn) {
    float r1 = pcg_next(smp);
    float r2 = pcg_next(smp);
    float alpha = 1 - sqrtf(r1);
    float beta = r2 * sqrtf(r1);
    float gamma = 1.0f - (alpha + beta);
    *pdf_pos = 1.0f / T->area;
    *p = vadd(vadd(vmuls(T->vx[0].p, alpha), vmuls(T->vx[1].p, beta)), vmuls(T->vx[2].p, gamma));
    float q2 = pcg_next(smp); /* cosineSampleHemisphere(sampler.next(), sampler.next()) */
    float q1 = pcg_next(smp);
    V3 wl = cosine_sample_hemisphere(q1, q2);
    *pdf_dir = (float)((wl.z >= 0.0f) ? (wl.z / O_PI) : 0.0f);
    *gn = vmuls(T->nrm, vdot(T->vx[0].n, T->nrm) > 0 ? 1.0f : -1.0f);
    Frame fr = frame_from(*gn);
    *wi = to_world(&fr, wl);
    (void)s;
}
/* RayTracer::lightTracePath (Renderer.h:292-326) */
static void light_trace_path(const struct or_scene* s, Ray* r, Col thr, Col Le, Pcg* smp, float* film, Counts* c) {
    for (;;) {
        Isect is = scene_traverse(s, r, c);
        Shading sd = shading_data(s, &is, r);
        if (!(sd.t < FLT_MAX)) return;
        if (is_light(sd.bsdf) || is_spec(sd.bsdf)) return;
        V3 wi = vnorm(vsub(v3(s->cam.origin[0], s->cam.origin[1], s->cam.origin[2]), sd.x));
        Col cl = cmul(cmul(thr, bsdf_eval(s, &sd)), Le);
        connect_to_camera(s, sd.x, sd.sN, cl, film, c);
        float rrp = win_min(clum(thr), 0.9f);
        if (pcg_next(smp) < rrp) thr = cdivs(thr, rrp);
        else return;
        Col ind;
        float pdf;
        V3 wi2 = bsdf_sample(s, &sd, smp, &ind, &pdf);
        thr = cdivs(cmuls(cmul(thr, ind), fabsf(vdot(wi2, sd.sN))), pdf);
        *r = ray_make(vadd(sd.x, vmuls(wi2, O_EPS)), wi2);
        (void)wi;
    }
}
/* RayTracer::lightTracer + lightTrace_init (Renderer.h:221-235, 264-291): W*H light paths per frame,
 * path i drawing from the PCG stream keyed (seed, i, frame). */
int or_render_light(or_scene* s, uint32_t first, uint32_t n_frames, uint64_t seed, float* film) {
    if (!s || !film || s->nlight <= 0) return -1;
    for (uint32_t f = first; f < first + n_frames; ++f) {
        for (uint32_t i = 0; i < (uint32_t)(s->W * s->H); ++i) {
            Pcg smp;
            pcg_init(&smp, seed, ((uint64_t)i << 16) | f);
            float pmf = 1.f / (float)s->nlight;
            int li = (int)((float)s->nlight * pcg_next(&smp));
            if (s->nlight - 1 < li) li = s->nlight - 1;
            int lt = s->light[li];
            if (lt < 0) continue; /* light->isArea() */
            const Tri* T = &s->tri[lt];
            V3 p, wi, gn;
            float pdf_pos, pdf_dir;
            light_emit_sample(s, T, &smp, &p, &pdf_pos, &wi, &pdf_dir, &gn);
            float cos_t = vdot(gn, wi);
            const float* e = s->mat[T->mat].emission;
            Col ev = vdot(vneg(wi), gn) < 0 ? col(e[0], e[1], e[2]) : col(0.0f, 0.0f, 0.0f); /* evaluate(-wi) */
            Col Le = cdivs(cmuls(ev, cos_t), (pmf * pdf_dir) * pdf_pos);
            connect_to_camera(s, p, gn, Le, film, NULL);
            Ray r = ray_make(p, wi);
            light_trace_path(s, &r, col(1.0f, 1.0f, 1.0f), Le, &smp, film, NULL);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ instant radiosity (Renderer.h:82-218) */
typedef struct { V3 x, n; Col Le; } Vpl;
typedef struct { Vpl* v; int n, cap; } VplList;
static void vpl_push(VplList* l, V3 x, V3 n, Col Le) {
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 64;
        l->v = (Vpl*)realloc(l->v, (size_t)l->cap * sizeof(Vpl));
    }
    l->v[l->n].x = x; l->v[l->n].n = n; l->v[l->n].Le = Le;
    l->n++;
}
/* RayTracer::VPLTracePath (Renderer.h:183-218, recursion unrolled) */
static void vpl_trace_path(const struct or_scene* s, Ray* r, Col thr, Col Le, Pcg* smp, VplList* out) {
    for (;;) {
        Isect is = scene_traverse(s, r, NULL);
        Shading sd = shading_data(s, &is, r);
        if (!(sd.t < FLT_MAX)) return;
        if (!is_light(sd.bsdf) && !is_spec(sd.bsdf))
            vpl_push(out, sd.x, sd.sN, cmuls(cmul(cmul(thr, Le), bsdf_eval(s, &sd)), fabsf(vdot(vneg(r->dir), sd.sN))));
        float rrp = win_min(clum(thr), 0.9f);
        if (pcg_next(smp) < rrp) thr = cdivs(thr, rrp);
        else return;
        Col val;
        float pdf;
        V3 wi = bsdf_sample(s, &sd, smp, &val, &pdf);
        thr = cdivs(cmuls(cmul(thr, val), fabsf(vdot(wi, sd.sN))), pdf);
        *r = ray_make(vadd(sd.x, vmuls(wi, O_EPS)), wi);
    }
}
/* RayTracer::instantRadiosity: traceVPLs (n_vpl paths, path i keyed (seed, i, frame)), then per pixel
 * the first hit and computeVPLsContribution (Renderer.h:101-156). */
int or_render_ir(or_scene* s, uint32_t first, uint32_t n_frames, uint64_t seed, uint32_t n_vpl, float* film) {
    if (!s || !film || s->nlight <= 0 || n_vpl == 0) return -1;
    for (uint32_t f = first; f < first + n_frames; ++f) {
        VplList vl = {NULL, 0, 0};
        for (uint32_t i = 0; i < n_vpl; ++i) {
            Pcg smp;
            pcg_init(&smp, seed, ((uint64_t)i << 16) | f);
            float pmf = 1.f / (float)s->nlight;
            int li = (int)((float)s->nlight * pcg_next(&smp));
            if (s->nlight - 1 < li) li = s->nlight - 1;
            int lt = s->light[li];
            if (lt < 0) continue;
            const Tri* T = &s->tri[lt];
            V3 p, wi, gn;
            float pdf_pos, pdf_dir;
            light_emit_sample(s, T, &smp, &p, &pdf_pos, &wi, &pdf_dir, &gn);
            const float* e = s->mat[T->mat].emission;
            Col ev = vdot(vneg(wi), gn) < 0 ? col(e[0], e[1], e[2]) : col(0.0f, 0.0f, 0.0f);
            float den = (pmf * pdf_pos) * (float)n_vpl;
            vpl_push(&vl, p, gn, cdivs(ev, den));
            Col Le = cdivs(cmuls(ev, vdot(wi, gn)), den);
            Ray r = ray_make(p, wi);
            vpl_trace_path(s, &r, col(1.0f, 1.0f, 1.0f), Le, &smp, &vl);
        }
        for (uint32_t y = 0; y < (uint32_t)s->H; ++y)
            for (uint32_t x = 0; x < (uint32_t)s->W; ++x) {
                Ray r = camera_ray(s, x + 0.5f, y + 0.5f);
                Isect is = scene_traverse(s, &r, NULL);
                Shading sd = shading_data(s, &is, &r);
                if (!(sd.t < FLT_MAX)) continue;
                Col sum = col(0.0f, 0.0f, 0.0f);
                if (!is_light(sd.bsdf) && !is_spec(sd.bsdf)) {
                    for (int j = 0; j < vl.n; ++j) {
                        V3 dir = vsub(vl.v[j].x, sd.x);
                        float dist2 = vlen2(dir);
                        if (dist2 < 1e-4f) continue;
                        dir = vnorm(dir);
                        float cv = vdot(vl.v[j].n, vneg(dir));
                        float cx = vdot(sd.sN, dir);
                        if (cv <= 0.0f || cx <= 0.0f) continue;
                        float G = (cv * cx) / dist2;
                        if (!scene_visible(s, sd.x, vl.v[j].x, NULL)) continue;
                        sum = cadd(sum, cmuls(cmul(vl.v[j].Le, bsdf_eval(s, &sd)), G));
                    }
                }
                splat(s, film, x + 0.5f, y + 0.5f, sum);
            }
        free(vl.v);
    }
    return 0;
}

/* Ray queries with the reference traversal (IntersectionData / Scene::visible semantics).
 * rays: n*8 (o.xyz, tmax, dir.xyz, pad); hits n*4 (t, id bits, alpha, beta). */
int or_trace_closest(or_scene* s, const float* rays, uint32_t n, float* hits) {
    for (uint32_t i = 0; i < n; ++i) {
        const float* q = rays + (size_t)i * 8;
        Ray r = ray_make(v3(q[0], q[1], q[2]), v3(q[4], q[5], q[6]));
        Isect is = scene_traverse(s, &r, NULL);
        int32_t id = is.t < FLT_MAX ? is.id : -1;
        hits[i * 4] = is.t;
        memcpy(&hits[i * 4 + 1], &id, 4);
        hits[i * 4 + 2] = is.t < FLT_MAX ? is.alpha : 0.0f;
        hits[i * 4 + 3] = is.t < FLT_MAX ? is.beta : 0.0f;
    }
    return 0;
}

int or_trace_visible(or_scene* s, const float* rays, uint32_t n, int32_t* vis) {
    for (uint32_t i = 0; i < n; ++i) {
        const float* q = rays + (size_t)i * 8;
        Ray r = ray_make(v3(q[0], q[1], q[2]), v3(q[4], q[5], q[6]));
        vis[i] = traverse_visible(s, 0, &r, q[3], NULL);
    }
    return 0;
}

/* Camera rays for pixel centres: out n*6 (o.xyz, dir.xyz). */
int or_camera_rays(or_scene* s, const uint32_t* pixels, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t x = pixels[i] % (uint32_t)s->W, y = pixels[i] / (uint32_t)s->W;
        Ray r = camera_ray(s, x + 0.5f, y + 0.5f);
        out[i * 6] = r.o.x; out[i * 6 + 1] = r.o.y; out[i * 6 + 2] = r.o.z;
        out[i * 6 + 3] = r.dir.x; out[i * 6 + 4] = r.dir.y; out[i * 6 + 5] = r.dir.z;
    }
    return 0;
}

/* Probes of the light-tracing pieces (tests): projectOntoCamera on points -> (ok, x, y); the
 * AreaLight emission sample of lights[li] from 4 scripted draws -> p, pdfPosition, wi, pdfDirection,
 * evaluate(-wi). */
int or_camera_project(or_scene* s, const float* pts, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; ++i) {
        float x = 0, y = 0;
        int ok = project_onto_camera(s, v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), &x, &y);
        out[3 * i] = ok ? 1.0f : 0.0f; out[3 * i + 1] = x; out[3 * i + 2] = y;
    }
    return 0;
}
int or_light_emit(or_scene* s, int li, const float* draws, float* out) {
    int lt = s->light[li];
    if (lt < 0) return -1;
    const Tri* T = &s->tri[lt];
    /* a stream whose next four draws are the scripted ones is not expressible with PCG: restate
     * the sampling here with the draws in call order (r1, r2, then the direction's q2, q1) */
    float r1 = draws[0], r2 = draws[1], q2 = draws[2], q1 = draws[3];
    float alpha = 1 - sqrtf(r1), beta = r2 * sqrtf(r1), gamma = 1.0f - (alpha + beta);
    V3 p = vadd(vadd(vmuls(T->vx[0].p, alpha), vmuls(T->vx[1].p, beta)), vmuls(T->vx[2].p, gamma));
    V3 wl = cosine_sample_hemisphere(q1, q2);
    V3 gn = vmuls(T->nrm, vdot(T->vx[0].n, T->nrm) > 0 ? 1.0f : -1.0f);
    Frame fr = frame_from(gn);
    V3 wi = to_world(&fr, wl);
    const float* e = s->mat[T->mat].emission;
    Col ev = vdot(vneg(wi), gn) < 0 ? col(e[0], e[1], e[2]) : col(0.0f, 0.0f, 0.0f);
    out[0] = p.x; out[1] = p.y; out[2] = p.z; out[3] = 1.0f / T->area;
    out[4] = wi.x; out[5] = wi.y; out[6] = wi.z; out[7] = (float)((wl.z >= 0.0f) ? (wl.z / O_PI) : 0.0f);
    out[8] = ev.r; out[9] = ev.g; out[10] = ev.b; out[11] = 4.0f;
    return 0;
}

/* Scalar probes of the shared math (for tests). */
float or_acosf(float x) { return O_ACOSF(x); }
float or_sinf(float x) { return O_SINF(x); }
float or_cosf(float x) { return O_COSF(x); }
float or_atan2f(float y, float x) { return O_ATAN2F(y, x); }
/* The flavour's transcendentals on arrays (fn as rtg_probe_math: 0 sinf, 1 cosf, 2 sincosf -> 2n
 * outputs, 3 acosf, 4 atan2f <- 2n inputs y, x): the libm build calls the C library. */
void or_math_eval(int fn, const float* in, uint32_t n, float* out)
{
    for (uint32_t i = 0; i < n; ++i) {
        switch (fn) {
        case 0: out[i] = O_SINF(in[i]); break;
        case 1: out[i] = O_COSF(in[i]); break;
#if ORACLE_LIBM
        case 2: sincosf(in[i], &out[2 * (size_t)i], &out[2 * (size_t)i + 1]); break;
#else
        case 2: rtm_sincosf(in[i], &out[2 * (size_t)i], &out[2 * (size_t)i + 1]); break;
#endif
        case 3: out[i] = O_ACOSF(in[i]); break;
        default: out[i] = O_ATAN2F(in[2 * (size_t)i], in[2 * (size_t)i + 1]); break;
        }
    }
}
/* rtm_sincosf (the GPU's fused form) against rtm_sinf / rtm_cosf on n inputs: number of inputs
 * whose bits differ in either result. */
long or_sincos_mismatch(const float* x, long n)
{
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        float s, c, s1 = rtm_sinf(x[i]), c1 = rtm_cosf(x[i]);
        rtm_sincosf(x[i], &s, &c);
        if (memcmp(&s, &s1, 4) != 0 || memcmp(&c, &c1, 4) != 0) ++bad;
    }
    return bad;
}
