// rtg_light.hip — the reference's two light-path integrators on the wavefront machinery of
// rtg_kernels.hip (k_trace for every ray query):
//
//   rtg_render_light               RayTracer::lightTracer / lightTrace_init / lightTracePath /
//                                  connectToCamera (RTBase/Renderer.h:221-326)
//   rtg_render_instant_radiosity   RayTracer::instantRadiosity / traceVPLs / VPLTracePath /
//                                  renderBlockinstantRadiosity / computeVPLsContribution
//                                  (RTBase/Renderer.h:82-218)
//
// Light tracing splats to whatever pixel a path vertex projects to. The reference runs all
// width*height light paths of a frame on one thread with one sampler, so a pixel receives its
// splats in (path, vertex) order. Here every visible camera connection becomes a record keyed
// (pixel << 40 | path << 16 | vertex); the records of a chunk are radix-sorted on the device
// (rocPRIM) and each pixel's run is added to the film in key order: the same additions in the
// same order, so the film is bit-identical to a sequential splat loop (oracle/rt_oracle.c).
//
// Instant radiosity: the VPL paths (a few dozen) are traced as a wavefront too, their VPLs are
// ordered by (path, vertex) as the reference's push_back order, and every pixel's first hit then
// tests every VPL (one any-hit ray per pixel x VPL, batched) and sums the contributions in VPL
// order.
//
// Sampler: path i of frame f draws from the PCG stream keyed (seed, i, f), the
// reference's single MTRandom being irreproducible across thread schedules anyway.
#include "rtg_internal.h"

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

struct DevProj {
    float P[16];    // projectionMatrix
    float C2V[16];  // cameraToView
    float vd[3];    // viewDirection
    float afilm;    // Afilm
    float ox, oy, oz, W, H;
};

// Camera::projectOntoCamera (Scene.h:55-69): cameraToView.mulPoint, then
// projectionMatrix.mulPointAndPerspectiveDivide (Core.h:302-320)
RTG_D bool project_onto_camera(const DevProj& c, v3 p, float& x, float& y) {
    const float* m = c.C2V;
    const v3 pv = mk(((p.x * m[0] + p.y * m[1]) + p.z * m[2]) + m[3], ((p.x * m[4] + p.y * m[5]) + p.z * m[6]) + m[7],
                     ((p.x * m[8] + p.y * m[9]) + p.z * m[10]) + m[11]);
    const float* q = c.P;
    const v3 v1 = mk(((pv.x * q[0] + pv.y * q[1]) + pv.z * q[2]) + q[3], ((pv.x * q[4] + pv.y * q[5]) + pv.z * q[6]) + q[7],
                     ((pv.x * q[8] + pv.y * q[9]) + pv.z * q[10]) + q[11]);
    float w = (((q[12] * pv.x) + (q[13] * pv.y)) + (q[14] * pv.z)) + q[15];
    w = 1.0f / w;
    const v3 pp = muls(v1, w);
    x = (pp.x + 1.0f) * 0.5f;
    y = (pp.y + 1.0f) * 0.5f;
    if (x < 0 || x > 1.0f || y < 0 || y > 1.0f) return false;
    x = x * c.W;
    y = 1.0f - y;
    y = y * c.H;
    return true;
}

// (int)x as x86-64 computes it (cvttss2si: NaN and out-of-range -> INT_MIN); gfx950's
// v_cvt_i32_f32 would give 0 for NaN
RTG_D int trunc_x86(float x) { return (x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : (int)0x80000000; }

// connectToCamera (Renderer.h:236-262) up to the visibility test: on success the splat pixel, the
// splatted colour col * W_e * G, and the Scene::visible(p, camera.origin) shadow ray.
RTG_D bool connect_to_camera(const DevProj& c, v3 p, v3 n, v3 col, int& pixel, v3& out, float4& so, float4& sd) {
    float x, y;
    if (!project_onto_camera(c, p, x, y)) return false;
    const v3 org = mk(c.ox, c.oy, c.oz);
    v3 dir = sub(org, p);
    const float dist2 = length_sq(dir);
    dir = normalize(dir);
    const float cs = dot(n, dir);
    const float cc = dot(mk(c.vd[0], c.vd[1], c.vd[2]), neg(dir));
    if (cs < 0.0f || cc < 0.0f) return false;
    const float G = (cs * cc) / dist2;
    const float We = 1 / (c.afilm * ((cc * cc) * (cc * cc)));  // SQ(SQ(cos_theta_cam))
    out = muls(muls(col, We), G);
    // Film::splat with the box filter of size 0 (Imaging.h:209-232): pixel ((int)x, (int)y) if inside
    const int px = trunc_x86(x), py = trunc_x86(y);
    if (!(px >= 0 && (unsigned)px < (unsigned)c.W && py >= 0 && (unsigned)py < (unsigned)c.H)) return false;
    pixel = py * (int)c.W + px;
    // Scene::visible(p, camera.origin) (Scene.h:161-169)
    v3 v = sub(org, p);
    const float maxt = sqrtf(length_sq(v)) - (2.0f * RTG_EPS);
    v = normalize(v);
    const v3 o = add(p, muls(v, RTG_EPS));
    so = make_float4(o.x, o.y, o.z, maxt);
    sd = make_float4(v.x, v.y, v.z, 0.0f);
    return true;
}

// Block-level compaction of up to two queues (ballot + mbcnt in a wave, LDS prefix over the waves,
// one atomic per queue per block). Every thread of the block must call it.
RTG_D void compact2(bool wa, bool wb, unsigned id, unsigned* qa, unsigned* na, unsigned* qb, unsigned* nb) {
    __shared__ unsigned cnt[2][RTG_TB / 64];
    __shared__ unsigned base[2];
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const unsigned long long ma = __ballot(wa), mb = __ballot(wb);
    if (lane == 0) {
        cnt[0][wave] = (unsigned)__popcll(ma);
        cnt[1][wave] = (unsigned)__popcll(mb);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned ta = 0, tb = 0;
        for (int w = 0; w < RTG_TB / 64; ++w) {
            ta += cnt[0][w];
            tb += cnt[1][w];
        }
        base[0] = ta ? atomicAdd(na, ta) : 0u;
        base[1] = tb ? atomicAdd(nb, tb) : 0u;
    }
    __syncthreads();
    unsigned oa = base[0], ob = base[1];
    for (int w = 0; w < wave; ++w) {
        oa += cnt[0][w];
        ob += cnt[1][w];
    }
    if (wa) qa[oa + prefix_lt(ma)] = id;
    if (wb) qb[ob + prefix_lt(mb)] = id;
}

struct LightArgs {
    unsigned base;        // global index of this chunk's path 0
    unsigned P;           // paths in the chunk
    unsigned sample;      // frame index (PCG stream key)
    unsigned long long seed;
    int vpl;              // 0: light tracer, 1: VPL paths (instant radiosity)
    float n_vpl;          // (float)N_VPLs
    DevProj cam;
};

// Light-path buffers (aliases of the path tracer's chunk buffers):
//   thr[pid] throughput, contrib[pid] (plane 0) the path's Le, rng[pid] PCG state,
//   ray_o/ray_d/hits extension ray, sh_o/sh_d camera-connection ray, sh_c its colour (.w = pixel bits),
//   meta[pid] any-hit visibility output.
// VPL records: rec_key[r] = path << 16 | vertex, rec[3r..3r+2] = (x, -), (sNormal, -), (Le, -).

// lightTrace_init (Renderer.h:264-291) / traceVPLs (:183-206): sample a light, a point and a
// direction on it; vertex 0 is the camera connection (light tracer) or the VPL on the light.
__global__ __launch_bounds__(RTG_TB) void k_light_generate(SceneView s, LightArgs a, PathBufs p, Counters* ctr,
                                                           unsigned long long* rec_key, float4* rec, unsigned* rec_n) {
    const unsigned pid = blockIdx.x * blockDim.x + threadIdx.x;
    bool want_ext = false, want_sh = false;
    if (pid < a.P) {
        const unsigned i = a.base + pid;
        const uint64_t inc = pcg_inc(i, a.sample);
        uint64_t st = pcg_seed(a.seed, inc);
        // Scene::sampleLight (Scene.h:131-140)
        const int nl = s.n_lights;
        const float pmf = s.pmf;  // 1.f / (float)nl
        int li = (int)((float)nl * pcg_next(st, inc));
        li = (nl - 1) < li ? (nl - 1) : li;
        const DevLight L = s.lights[li];
        if (__float_as_int(L.v1t.w) == 0) {  // light->isArea()
            // samplePositionFromLight -> Triangle::sample (Geometry.h:114-126)
            const float r1 = pcg_next(st, inc);
            const float r2 = pcg_next(st, inc);
            const float la = 1 - sqrtf(r1);
            const float lb = r2 * sqrtf(r1);
            const float lg = 1.0f - (la + lb);
            const float pdf_pos = L.v2.w;  // 1.0f / area
            const v3 pt = add(add(muls(mk(L.v0a.x, L.v0a.y, L.v0a.z), la), muls(mk(L.v1t.x, L.v1t.y, L.v1t.z), lb)),
                              muls(mk(L.v2.x, L.v2.y, L.v2.z), lg));
            // sampleDirectionFromLight (Lights.h:67-80): cosineSampleHemisphere(next(), next()), first draw -> r2
            const float q2 = pcg_next(st, inc);
            const float q1 = pcg_next(st, inc);
            const v3 wl = cosine_sample_hemisphere(q1, q2);
            const float pdf_dir = (wl.z >= 0.0f) ? div_pi_d(wl.z) : 0.0f;
            const v3 gn = mk(L.gn.x, L.gn.y, L.gn.z);
            const frame fr = frame_from(gn);
            const v3 wi = to_world(fr, wl);
            // AreaLight::evaluate(-wi) (Lights.h:40-47)
            const v3 ev = dot(neg(wi), gn) < 0 ? mk(L.em.x, L.em.y, L.em.z) : mk(0.0f, 0.0f, 0.0f);
            v3 le;
            if (!a.vpl) {
                const float cos_t = dot(gn, wi);
                le = divs(muls(ev, cos_t), (pmf * pdf_dir) * pdf_pos);
                int pixel;
                v3 cc;
                float4 so, sd;
                if (connect_to_camera(a.cam, pt, gn, le, pixel, cc, so, sd)) {
                    p.sh_o[pid] = so;
                    p.sh_d[pid] = sd;
                    p.sh_c[pid] = make_float4(cc.x, cc.y, cc.z, __int_as_float(pixel));
                    want_sh = true;
                }
            } else {
                // the VPL on the light: ShadingData(p, n), Le = evaluate(-wi) / (pmf * pdfPosition * N)
                const float den = (pmf * pdf_pos) * a.n_vpl;
                const v3 vle = divs(ev, den);
                const unsigned r = atomicAdd(rec_n, 1u);
                rec_key[r] = ((unsigned long long)i << 16);
                rec[3 * r + 0] = make_float4(pt.x, pt.y, pt.z, 0.0f);
                rec[3 * r + 1] = make_float4(gn.x, gn.y, gn.z, 0.0f);
                rec[3 * r + 2] = make_float4(vle.x, vle.y, vle.z, 0.0f);
                le = divs(muls(ev, dot(wi, gn)), den);
            }
            p.contrib[pid] = make_float4(le.x, le.y, le.z, 0.0f);
            p.thr[pid] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
            p.ray_o[pid] = make_float4(pt.x, pt.y, pt.z, 0.0f);  // Ray(p, wi): no offset
            p.ray_d[pid] = make_float4(wi.x, wi.y, wi.z, 0.0f);
            p.rng[pid] = st;
            want_ext = true;
        }
    }
    compact2(want_ext, want_sh, pid, p.q[0], &ctr->n_ext, p.shq, &ctr->n_shadow);
}

// lightTracePath (Renderer.h:292-326) / VPLTracePath (:207-218) at vertex k >= 1 (the hit of the
// extension ray of vertex k-1). qin / n: extension queue of the previous vertex.
__global__ __launch_bounds__(RTG_TB) void k_light_shade(SceneView s, LightArgs a, PathBufs p, const unsigned* qin,
                                                        unsigned n, unsigned* qout, Counters* ctr, unsigned k,
                                                        unsigned long long* rec_key, float4* rec, unsigned* rec_n) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    bool want_ext = false, want_sh = false;
    unsigned pid = 0;
    if (t < n) {
        pid = qin[t];
        const float4 h = p.hits[pid];
        if (h.x < RTG_FLT_MAX) {
            const float4 ro = p.ray_o[pid], rd = p.ray_d[pid];
            const v3 o = mk(ro.x, ro.y, ro.z), d = mk(rd.x, rd.y, rd.z);
            const float4 thr4 = p.thr[pid], le4 = p.contrib[pid];
            v3 thr = mk(thr4.x, thr4.y, thr4.z);
            const v3 le = mk(le4.x, le4.y, le4.z);
            // Scene::calculateShadingData (Scene.h:174-203)
            const int tri = __float_as_int(h.y);
            const float alpha = h.z, beta = h.w, gamma = 1.0f - (alpha + beta);
            const v3 x = add(o, muls(d, h.x));
            const DevShade S = s.shade[tri];
            const DevMat M = s.mats[__float_as_int(S.d.w)];
            const v3 n0 = mk(S.a.x, S.a.y, S.a.z), n1 = mk(S.a.w, S.b.x, S.b.y), n2 = mk(S.b.z, S.b.w, S.c.x);
            v3 sn = normalize(add(add(muls(n0, alpha), muls(n1, beta)), muls(n2, gamma)));
            const float tu = (S.c.y * alpha + S.c.w * beta) + S.d.y * gamma;
            const float tv = (S.c.z * alpha + S.d.x * beta) + S.d.z * gamma;
            const v3 wo = neg(d);
            if (M.two_sided && dot(wo, sn) < 0) sn = neg(sn);
            const frame fr = frame_from(sn);
            const bool spec = M.kind == RTG_MAT_MIRROR || M.kind == RTG_MAT_GLASS;
            const unsigned i = a.base + pid;
            const uint64_t inc = pcg_inc(i, a.sample);
            uint64_t st = p.rng[pid];
            bool cont = true;
            if (!a.vpl) {
                if (M.is_light || spec) {
                    cont = false;  // lightTracePath returns at lights and pure specular surfaces
                } else {
                    const v3 f = divs_pi(tex_sample(s, M, tu, tv));  // BSDF::evaluate
                    const v3 col = mul(mul(thr, f), le);
                    int pixel;
                    v3 cc;
                    float4 so, sd;
                    if (connect_to_camera(a.cam, x, sn, col, pixel, cc, so, sd)) {
                        p.sh_o[pid] = so;
                        p.sh_d[pid] = sd;
                        p.sh_c[pid] = make_float4(cc.x, cc.y, cc.z, __int_as_float(pixel));
                        want_sh = true;
                    }
                }
            } else if (!M.is_light && !spec) {
                // store a VPL: Le = pathThroughput * Le * evaluate(sd, -r.dir) * |(-r.dir) . sN|
                const v3 f = divs_pi(tex_sample(s, M, tu, tv));
                const v3 vle = muls(mul(mul(thr, le), f), fabsf(dot(wo, sn)));
                const unsigned r = atomicAdd(rec_n, 1u);
                rec_key[r] = ((unsigned long long)i << 16) | k;
                rec[3 * r + 0] = make_float4(x.x, x.y, x.z, 0.0f);
                rec[3 * r + 1] = make_float4(sn.x, sn.y, sn.z, 0.0f);
                rec[3 * r + 2] = make_float4(vle.x, vle.y, vle.z, 0.0f);
            }
            if (cont) {
                const float rrp = wmin(lum(thr), 0.9f);
                if (pcg_next(st, inc) < rrp) {
                    thr = divs(thr, rrp);
                    v3 ind;
                    float pdf;
                    PcgSampler smp{st, inc};
                    const v3 wi = bsdf_sample(M.kind, M.int_ior, M.ext_ior, tex_sample(s, M, tu, tv), fr, wo, smp,
                                              ind, pdf);
                    st = smp.s;
                    thr = divs(muls(mul(thr, ind), fabsf(dot(wi, sn))), pdf);
                    const v3 no = add(x, muls(wi, RTG_EPS));
                    p.ray_o[pid] = make_float4(no.x, no.y, no.z, 0.0f);
                    p.ray_d[pid] = make_float4(wi.x, wi.y, wi.z, 0.0f);
                    p.thr[pid] = make_float4(thr.x, thr.y, thr.z, 0.0f);
                    p.rng[pid] = st;
                    want_ext = true;
                }
            }
        }
    }
    compact2(want_ext, want_sh, pid, qout, &ctr->n_ext, p.shq, &ctr->n_shadow);
}

// Visible camera connections of vertex k -> splat records (key, colour).
__global__ __launch_bounds__(RTG_TB) void k_light_collect(LightArgs a, PathBufs p, unsigned n, unsigned k,
                                                          unsigned long long* key, float4* col, unsigned* rec_n) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const unsigned pid = p.shq[t];
    if (!p.meta[pid]) return;
    const float4 c = p.sh_c[pid];
    const unsigned pixel = (unsigned)__float_as_int(c.w);
    const unsigned r = atomicAdd(rec_n, 1u);
    key[r] = ((unsigned long long)pixel << 40) | ((unsigned long long)(a.base + pid) << 16) | k;
    col[r] = make_float4(c.x, c.y, c.z, 0.0f);
}

// Film::splat in key order: one thread per pixel run of the sorted records.
__global__ __launch_bounds__(RTG_TB) void k_light_splat(const unsigned long long* key, const unsigned* idx,
                                                        const float4* col, unsigned n, float* film) {
    const unsigned r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const unsigned long long pix = key[r] >> 40;
    if (r > 0 && (key[r - 1] >> 40) == pix) return;
    float* f = film + (size_t)pix * 3;
    float fr = f[0], fg = f[1], fb = f[2];
    for (unsigned j = r; j < n && (key[j] >> 40) == pix; ++j) {
        const float4 c = col[idx[j]];
        // film[i] + (L * filterWeight / total) with weight = total = 1 (BoxFilter, size 0)
        fr = fr + ((c.x * 1.0f) / 1.0f);
        fg = fg + ((c.y * 1.0f) / 1.0f);
        fb = fb + ((c.z * 1.0f) / 1.0f);
    }
    f[0] = fr;
    f[1] = fg;
    f[2] = fb;
}

__global__ void k_iota(unsigned* v, unsigned n) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// ---- instant radiosity: per-pixel first hit (renderBlockinstantRadiosity, Renderer.h:83-100)
// px[lp] = (x, flag) with flag 0 = miss (no splat), 1 = hit on a light or pure specular surface
// (contribution 0), 2 = contributes; pn[lp] = (sNormal, -); pf[lp] = (BSDF::evaluate, -);
// acc[lp] = running VPL sum.
__global__ __launch_bounds__(RTG_TB) void k_ir_first_hit(SceneView s, ChunkArgs a, PathBufs p, float4* px, float4* pn,
                                                         float4* pf, float4* acc) {
    const unsigned lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= a.npix) return;
    const float4 h = p.hits[lp];
    float flag = 0.0f;
    v3 x = mk(0.0f, 0.0f, 0.0f), sn = x, f = x;
    if (h.x < RTG_FLT_MAX) {
        const float4 ro = p.ray_o[lp], rd = p.ray_d[lp];
        const v3 o = mk(ro.x, ro.y, ro.z), d = mk(rd.x, rd.y, rd.z);
        const int tri = __float_as_int(h.y);
        const float alpha = h.z, beta = h.w, gamma = 1.0f - (alpha + beta);
        x = add(o, muls(d, h.x));
        const DevShade S = s.shade[tri];
        const DevMat M = s.mats[__float_as_int(S.d.w)];
        const v3 n0 = mk(S.a.x, S.a.y, S.a.z), n1 = mk(S.a.w, S.b.x, S.b.y), n2 = mk(S.b.z, S.b.w, S.c.x);
        sn = normalize(add(add(muls(n0, alpha), muls(n1, beta)), muls(n2, gamma)));
        const float tu = (S.c.y * alpha + S.c.w * beta) + S.d.y * gamma;
        const float tv = (S.c.z * alpha + S.d.x * beta) + S.d.z * gamma;
        if (M.two_sided && dot(neg(d), sn) < 0) sn = neg(sn);
        const bool spec = M.kind == RTG_MAT_MIRROR || M.kind == RTG_MAT_GLASS;
        flag = (M.is_light || spec) ? 1.0f : 2.0f;
        if (!M.is_light && !spec) f = divs_pi(tex_sample(s, M, tu, tv));
    }
    px[lp] = make_float4(x.x, x.y, x.z, flag);
    pn[lp] = make_float4(sn.x, sn.y, sn.z, 0.0f);
    pf[lp] = make_float4(f.x, f.y, f.z, 0.0f);
    acc[lp] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// computeVPLsContribution (Renderer.h:125-156), geometry part: the shadow rays of VPLs [j0, j0+nb)
__global__ __launch_bounds__(RTG_TB) void k_ir_rays(unsigned npix, const float4* px, const float4* pn, const float4* vpl,
                                                    unsigned j0, unsigned nb, float4* so, float4* sd, unsigned* q,
                                                    unsigned* qn) {
    const unsigned r = blockIdx.x * blockDim.x + threadIdx.x;
    bool want = false;
    if (r < npix * nb) {
        const unsigned lp = r / nb, j = j0 + r % nb;
        const float4 X = px[lp];
        if (X.w == 2.0f) {
            const float4 N = pn[lp], V = vpl[3 * j], VN = vpl[3 * j + 1];
            const v3 x = mk(X.x, X.y, X.z), vx = mk(V.x, V.y, V.z);
            v3 dir = sub(vx, x);
            const float dist2 = length_sq(dir);
            if (!(dist2 < 1e-4f)) {
                dir = normalize(dir);
                const float cv = dot(mk(VN.x, VN.y, VN.z), neg(dir));
                const float cx = dot(mk(N.x, N.y, N.z), dir);
                if (!(cv <= 0.0f || cx <= 0.0f)) {
                    v3 v = sub(vx, x);  // Scene::visible(shadingData.x, vpl.x)
                    const float maxt = sqrtf(length_sq(v)) - (2.0f * RTG_EPS);
                    v = normalize(v);
                    const v3 o = add(x, muls(v, RTG_EPS));
                    so[r] = make_float4(o.x, o.y, o.z, maxt);
                    sd[r] = make_float4(v.x, v.y, v.z, 0.0f);
                    want = true;
                }
            }
        }
    }
    compact2(want, false, r, q, qn, q, qn);
}

// computeVPLsContribution, shading part: col_sum += vpl.Le * bsdf * G over visible VPLs, in order
__global__ __launch_bounds__(RTG_TB) void k_ir_accumulate(unsigned npix, const float4* px, const float4* pn,
                                                          const float4* pf, const float4* vpl, unsigned j0, unsigned nb,
                                                          const int* vis, float4* acc) {
    const unsigned lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= npix) return;
    const float4 X = px[lp];
    if (X.w != 2.0f) return;
    const float4 N = pn[lp], F = pf[lp];
    float4 A = acc[lp];
    const v3 x = mk(X.x, X.y, X.z), sn = mk(N.x, N.y, N.z), f = mk(F.x, F.y, F.z);
    v3 sum = mk(A.x, A.y, A.z);
    for (unsigned jj = 0; jj < nb; ++jj) {
        if (!vis[(size_t)lp * nb + jj]) continue;
        const unsigned j = j0 + jj;
        const float4 V = vpl[3 * j], VN = vpl[3 * j + 1], VL = vpl[3 * j + 2];
        v3 dir = sub(mk(V.x, V.y, V.z), x);
        const float dist2 = length_sq(dir);
        dir = normalize(dir);
        const float cv = dot(mk(VN.x, VN.y, VN.z), neg(dir));
        const float cx = dot(sn, dir);
        const float G = (cv * cx) / dist2;
        const v3 c = muls(mul(mk(VL.x, VL.y, VL.z), f), G);
        sum = add(sum, c);
    }
    acc[lp] = make_float4(sum.x, sum.y, sum.z, 0.0f);
}

// film->splat(x, y, col) for pixels whose camera ray hit something
__global__ __launch_bounds__(RTG_TB) void k_ir_splat(const unsigned* pixlist, unsigned npix, const float4* px,
                                                     const float4* acc, float* film) {
    const unsigned lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= npix || px[lp].w == 0.0f) return;
    const float4 c = acc[lp];
    float* f = film + (size_t)pixlist[lp] * 3;
    f[0] = f[0] + ((c.x * 1.0f) / 1.0f);
    f[1] = f[1] + ((c.y * 1.0f) / 1.0f);
    f[2] = f[2] + ((c.z * 1.0f) / 1.0f);
}

// ------------------------------------------------------------------ host helpers
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { (void)hipFree(p); }
    template <class T>
    T* get() { return (T*)p; }
};
#define DALLOC(buf, bytes) HIPOK(hipMalloc(&(buf).p, std::max<size_t>((bytes), 16)))

static DevProj make_proj(const rtg_handle* h) {
    DevProj c;
    std::memcpy(c.P, h->proj.proj, sizeof(c.P));
    std::memcpy(c.C2V, h->proj.camera_to_view, sizeof(c.C2V));
    std::memcpy(c.vd, h->proj.view_direction, sizeof(c.vd));
    c.afilm = h->proj.a_film;
    c.ox = h->cam.ox;
    c.oy = h->cam.oy;
    c.oz = h->cam.oz;
    c.W = h->cam.width;
    c.H = h->cam.height;
    return c;
}

static unsigned grid(size_t n) { return (unsigned)std::max<size_t>(1, (n + RTG_TB - 1) / RTG_TB); }

static int read_ctr(Counters* d, Counters& out, hipStream_t st) {
    HIPOK(hipMemcpyAsync(&out, d, sizeof(Counters), hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    return RTG_OK;
}

// Light-path wavefront for paths [base, base+P) of frame `sample`. Light tracer (vpl = 0): splat
// records into key/col (count in *rec_n, capacity cap); VPL mode: VPL records.
static int trace_light_paths(rtg_handle* h, hipStream_t st, LightArgs& a, PathBufs& pb, unsigned long long* key,
                             float4* col, unsigned* d_rec_n, size_t cap) {
    TraceIO io{};
    io.stats = h->d_stats;
    io.cull = h->cull;
    io.wide = h->wide;
    io.ovf = h->slot[0].d_ovf;
    io.ray_o = pb.ray_o;
    io.ray_d = pb.ray_d;
    io.hits = pb.hits;
    io.squeue = pb.shq;
    io.sray_o = pb.sh_o;
    io.sray_d = pb.sh_d;
    io.visible = pb.meta;
    HIPOK(hipMemsetAsync(pb.ctr, 0, 2 * sizeof(Counters), st));
    hipLaunchKernelGGL(k_light_generate, dim3(grid(a.P)), dim3(RTG_TB), 0, st, h->sv, a, pb, pb.ctr, key, col, d_rec_n);
    LAUNCH_OK("k_light_generate");
    h->stats.paths += a.P;
    for (unsigned k = 0;; ++k) {
        const int c = k & 1;
        Counters cn;
        int rc = read_ctr(pb.ctr + c, cn, st);
        if (rc) return rc;
        unsigned rn = 0;
        HIPOK(hipMemcpy(&rn, d_rec_n, sizeof(unsigned), hipMemcpyDeviceToHost));
        if ((size_t)rn + cn.n_shadow + cn.n_ext > cap) { g_err = "light tracing: record buffer overflow"; return RTG_ERR_HIP; }
        if (cn.n_ext == 0 && cn.n_shadow == 0) break;
        if (k >= 65535) { g_err = "light path longer than 65535 vertices"; return RTG_ERR_ARG; }
        h->stats.extension_rays += cn.n_ext;
        h->stats.shadow_rays += cn.n_shadow;
        // trace: extension rays of vertex k and camera connections of vertex k
        io.queue = pb.q[c];
        io.count = &pb.ctr[c].n_ext;
        io.scount = &pb.ctr[c].n_shadow;
        io.fetch = &pb.ctr[c].f_ext;
        if ((rc = launch_trace(h, io, st))) return rc;
        if (!a.vpl && cn.n_shadow) {
            hipLaunchKernelGGL(k_light_collect, dim3(grid(cn.n_shadow)), dim3(RTG_TB), 0, st, a, pb, cn.n_shadow, k, key,
                               col, d_rec_n);
            LAUNCH_OK("k_light_collect");
        }
        HIPOK(hipMemsetAsync(pb.ctr + (c ^ 1), 0, sizeof(Counters), st));
        if (cn.n_ext) {
            hipLaunchKernelGGL(k_light_shade, dim3(grid(cn.n_ext)), dim3(RTG_TB), 0, st, h->sv, a, pb, pb.q[c], cn.n_ext,
                               pb.q[c ^ 1], pb.ctr + (c ^ 1), k + 1, key, col, d_rec_n);
            LAUNCH_OK("k_light_shade");
        }
    }
    return RTG_OK;
}

}  // namespace

extern "C" {

int rtg_render_light(rtg_handle* h, uint32_t first, uint32_t n_frames, uint64_t seed) {
    if (!h) { g_err = "rtg_render_light: null handle"; return RTG_ERR_ARG; }
    HIPOK(hipSetDevice(h->device));
    hipStream_t st = h->stream;
    const size_t npaths = (size_t)h->W * h->H;  // lightTracer: one light path per pixel of the film
    if (npaths >= (1ull << 24)) { g_err = "rtg_render_light: film larger than 2^24 pixels (record key)"; return RTG_ERR_ARG; }
    if ((uint64_t)first + n_frames > 65536u) { g_err = "frame index >= 65536 (PCG stream key)"; return RTG_ERR_ARG; }
    const size_t P = std::min<size_t>(npaths, h->max_paths);
    int rc;
    if ((rc = join_frames(h))) return rc;
    HIPOK(hipStreamSynchronize(st));  // slot 0's buffers are free
    if ((rc = ensure_chunk(h, h->slot[0], P, std::max(h->slot[0].cap_maxb, 1), true))) return rc;
    if ((rc = ensure_ovf(h, h->slot[0]))) return rc;
    // records: at most one per path and vertex; grown on demand
    size_t cap = 4 * P + 1024;
    DevBuf key, col, key2, idx, idx2, rn, tmp;
    DALLOC(key, cap * 8); DALLOC(col, cap * 16); DALLOC(key2, cap * 8); DALLOC(idx, cap * 4); DALLOC(idx2, cap * 4);
    DALLOC(rn, 16);
    size_t tmp_bytes = 0;
    const DevProj cam = make_proj(h);
    PathBufs& pb = h->slot[0].pb;
    for (uint32_t f = first; f < first + n_frames; ++f) {
        for (size_t base = 0; base < npaths; base += P) {
            LightArgs a{};
            a.base = (unsigned)base;
            a.P = (unsigned)std::min(P, npaths - base);
            a.sample = f;
            a.seed = seed;
            a.vpl = 0;
            a.cam = cam;
            HIPOK(hipMemsetAsync(rn.p, 0, 16, st));
            for (;;) {  // grow the record buffers if a chunk overflows them (rare), then retry it
                rc = trace_light_paths(h, st, a, pb, key.get<unsigned long long>(), col.get<float4>(), rn.get<unsigned>(), cap);
                if (rc == RTG_OK) break;
                if (g_err != "light tracing: record buffer overflow") return rc;
                cap *= 4;
                (void)hipFree(key.p); (void)hipFree(col.p); (void)hipFree(key2.p); (void)hipFree(idx.p); (void)hipFree(idx2.p);
                key.p = col.p = key2.p = idx.p = idx2.p = nullptr;
                DALLOC(key, cap * 8); DALLOC(col, cap * 16); DALLOC(key2, cap * 8); DALLOC(idx, cap * 4); DALLOC(idx2, cap * 4);
                HIPOK(hipMemsetAsync(rn.p, 0, 16, st));
            }
            unsigned n = 0;
            HIPOK(hipMemcpyAsync(&n, rn.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
            HIPOK(hipStreamSynchronize(st));
            if (n == 0) continue;
            hipLaunchKernelGGL(k_iota, dim3(grid(n)), dim3(RTG_TB), 0, st, idx.get<unsigned>(), n);
            LAUNCH_OK("k_iota");
            size_t need = 0;
            HIPOK(rocprim::radix_sort_pairs(nullptr, need, key.get<unsigned long long>(), key2.get<unsigned long long>(),
                                            idx.get<unsigned>(), idx2.get<unsigned>(), n, 0, 64, st));
            if (need > tmp_bytes) {
                (void)hipFree(tmp.p);
                tmp.p = nullptr;
                DALLOC(tmp, need);
                tmp_bytes = need;
            }
            HIPOK(rocprim::radix_sort_pairs(tmp.p, need, key.get<unsigned long long>(), key2.get<unsigned long long>(),
                                            idx.get<unsigned>(), idx2.get<unsigned>(), n, 0, 64, st));
            hipLaunchKernelGGL(k_light_splat, dim3(grid(n)), dim3(RTG_TB), 0, st, key2.get<unsigned long long>(),
                               idx2.get<unsigned>(), (const float4*)col.p, n, h->d_film);
            LAUNCH_OK("k_light_splat");
        }
        h->spp += 1;  // render(): film->incrementSPP()
    }
    HIPOK(hipStreamSynchronize(st));
    return RTG_OK;
}

int rtg_render_instant_radiosity(rtg_handle* h, uint32_t first, uint32_t n_frames, uint64_t seed, uint32_t n_vpl) {
    if (!h || n_vpl == 0) { g_err = "rtg_render_instant_radiosity: bad argument"; return RTG_ERR_ARG; }
    HIPOK(hipSetDevice(h->device));
    hipStream_t st = h->stream;
    if ((uint64_t)first + n_frames > 65536u) { g_err = "frame index >= 65536 (PCG stream key)"; return RTG_ERR_ARG; }
    int rc;
    if ((rc = join_frames(h))) return rc;
    HIPOK(hipStreamSynchronize(st));  // slot 0's buffers are free
    if ((rc = set_pixels(h, nullptr, 0))) return rc;
    const unsigned npix = h->npix;
    if ((rc = ensure_chunk(h, h->slot[0], std::max<size_t>(npix, n_vpl), std::max(h->slot[0].cap_maxb, 1), true))) return rc;
    if ((rc = ensure_ovf(h, h->slot[0]))) return rc;
    PathBufs& pb = h->slot[0].pb;
    const DevProj cam = make_proj(h);
    size_t cap = 64 * (size_t)n_vpl + 1024;
    DevBuf vkey, vrec, rn, px, pn, pf, acc, vpl_d;
    DALLOC(vkey, cap * 8); DALLOC(vrec, cap * 48); DALLOC(rn, 16);
    DALLOC(px, (size_t)npix * 16); DALLOC(pn, (size_t)npix * 16); DALLOC(pf, (size_t)npix * 16); DALLOC(acc, (size_t)npix * 16);
    for (uint32_t f = first; f < first + n_frames; ++f) {
        // ---- traceVPLs (Renderer.h:183-206)
        LightArgs a{};
        a.base = 0;
        a.P = n_vpl;
        a.sample = f;
        a.seed = seed;
        a.vpl = 1;
        a.n_vpl = (float)n_vpl;
        a.cam = cam;
        for (;;) {
            HIPOK(hipMemsetAsync(rn.p, 0, 16, st));
            rc = trace_light_paths(h, st, a, pb, vkey.get<unsigned long long>(), vrec.get<float4>(), rn.get<unsigned>(), cap);
            if (rc == RTG_OK) break;
            if (g_err != "light tracing: record buffer overflow") return rc;
            cap *= 4;
            (void)hipFree(vkey.p); (void)hipFree(vrec.p);
            vkey.p = vrec.p = nullptr;
            DALLOC(vkey, cap * 8); DALLOC(vrec, cap * 48);
        }
        unsigned nv = 0;
        HIPOK(hipMemcpy(&nv, rn.p, sizeof(unsigned), hipMemcpyDeviceToHost));
        // VPL list in the reference's push_back order: by (path, vertex)
        std::vector<unsigned long long> hk(nv);
        std::vector<float4> hr((size_t)nv * 3), vl((size_t)std::max(nv, 1u) * 3);
        if (nv) {
            HIPOK(hipMemcpy(hk.data(), vkey.p, (size_t)nv * 8, hipMemcpyDeviceToHost));
            HIPOK(hipMemcpy(hr.data(), vrec.p, (size_t)nv * 48, hipMemcpyDeviceToHost));
        }
        std::vector<unsigned> order(nv);
        for (unsigned i = 0; i < nv; ++i) order[i] = i;
        std::sort(order.begin(), order.end(), [&](unsigned x, unsigned y) { return hk[x] < hk[y]; });
        for (unsigned i = 0; i < nv; ++i)
            for (int c = 0; c < 3; ++c) vl[3 * i + c] = hr[3 * (size_t)order[i] + c];
        (void)hipFree(vpl_d.p);
        vpl_d.p = nullptr;
        DALLOC(vpl_d, vl.size() * 16);
        HIPOK(hipMemcpy(vpl_d.p, vl.data(), vl.size() * 16, hipMemcpyHostToDevice));
        // ---- camera rays and first hits (renderBlockinstantRadiosity, Renderer.h:83-100)
        ChunkArgs ca{};
        ca.pixlist = h->d_pix;
        ca.npix = npix;
        ca.ns = 1;
        ca.s0 = f;
        ca.P = npix;
        ca.seed = seed;
        ca.max_depth = h->max_depth;
        ca.mode = RTG_INTEGRATOR_PATH;
        ca.cam = h->cam;
        HIPOK(hipMemsetAsync(pb.ctr, 0, 2 * sizeof(Counters), st));
        if ((rc = launch_generate(h, ca, pb, st))) return rc;
        TraceIO io{};
        io.stats = h->d_stats;
        io.cull = h->cull;
        io.wide = h->wide;
        io.ovf = h->slot[0].d_ovf;
        io.queue = pb.q[0];
        io.ray_o = pb.ray_o;
        io.ray_d = pb.ray_d;
        io.count = &pb.ctr[0].n_ext;
        io.hits = pb.hits;
        io.fetch = &pb.ctr[0].f_ext;
        if ((rc = launch_trace(h, io, st))) return rc;
        h->stats.extension_rays += npix;
        h->stats.paths += npix;
        hipLaunchKernelGGL(k_ir_first_hit, dim3(grid(npix)), dim3(RTG_TB), 0, st, h->sv, ca, pb, px.get<float4>(),
                           pn.get<float4>(), pf.get<float4>(), acc.get<float4>());
        LAUNCH_OK("k_ir_first_hit");
        // ---- every pixel x every VPL, in VPL batches (computeVPLsContribution, Renderer.h:125-156)
        if (nv) {
            const unsigned nb = (unsigned)std::max<size_t>(1, std::min<size_t>(nv, h->max_paths / std::max(1u, npix)));
            const size_t R = (size_t)npix * nb;
            DevBuf so, sd, q, vis, qn;
            DALLOC(so, R * 16); DALLOC(sd, R * 16); DALLOC(q, R * 4); DALLOC(vis, R * 4); DALLOC(qn, 16);
            for (unsigned j0 = 0; j0 < nv; j0 += nb) {
                const unsigned b = std::min(nb, nv - j0);
                const size_t Rb = (size_t)npix * b;
                HIPOK(hipMemsetAsync(qn.p, 0, 16, st));
                HIPOK(hipMemsetAsync(vis.p, 0, Rb * 4, st));
                hipLaunchKernelGGL(k_ir_rays, dim3(grid(Rb)), dim3(RTG_TB), 0, st, npix, (const float4*)px.p,
                                   (const float4*)pn.p, (const float4*)vpl_d.p, j0, b, so.get<float4>(), sd.get<float4>(),
                                   q.get<unsigned>(), qn.get<unsigned>());
                LAUNCH_OK("k_ir_rays");
                TraceIO sio{};
                sio.stats = h->d_stats;
                sio.cull = h->cull;
                sio.wide = h->wide;
                sio.ovf = h->slot[0].d_ovf;
                sio.squeue = q.get<unsigned>();
                sio.sray_o = so.get<float4>();
                sio.sray_d = sd.get<float4>();
                sio.scount = qn.get<unsigned>();
                sio.visible = vis.get<int>();
                sio.fetch = qn.get<unsigned>() + 1;
                if ((rc = launch_trace(h, sio, st))) return rc;
                hipLaunchKernelGGL(k_ir_accumulate, dim3(grid(npix)), dim3(RTG_TB), 0, st, npix, (const float4*)px.p,
                                   (const float4*)pn.p, (const float4*)pf.p, (const float4*)vpl_d.p, j0, b,
                                   (const int*)vis.p, acc.get<float4>());
                LAUNCH_OK("k_ir_accumulate");
                unsigned ns = 0;
                HIPOK(hipMemcpyAsync(&ns, qn.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
                HIPOK(hipStreamSynchronize(st));
                h->stats.shadow_rays += ns;
            }
        }
        hipLaunchKernelGGL(k_ir_splat, dim3(grid(npix)), dim3(RTG_TB), 0, st, (const unsigned*)h->d_pix, npix,
                           (const float4*)px.p, (const float4*)acc.p, h->d_film);
        LAUNCH_OK("k_ir_splat");
        h->spp += 1;
    }
    HIPOK(hipStreamSynchronize(st));
    return RTG_OK;
}

}  // extern "C"
