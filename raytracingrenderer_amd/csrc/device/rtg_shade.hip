// rtg_shade.hip — k_shade, the shading stage of the wavefront path tracer (see rtg_kernels.hip's
// header for the bounce loop), in a translation unit of its own so that it can be compiled with its
// own instruction-scheduling strategy (raytracingrenderer_amd/build.py: SHADE_FLAGS).
#include "rtg_internal.h"

#include <hip/hip_runtime.h>

// ------------------------------------------------------------------ shade
// Path state travels with the queues: the extension payload of bounce b (origin with the path id
// in .w, direction with canHitLight in .w, throughput, PCG state) sits at the ray's position in
// the extension queue, in buffer set b & 1. k_trace and k_shade read it by position (contiguous, no
// id -> payload indirection in either kernel's dependent chain); k_shade writes a continuing
// path's next payload at its position in set (b + 1) & 1 and an NEE ray (staged in LDS: held in
// registers across the BSDF sample it spilled) at its shadow-queue position, the path id beside
// it. Per-path results (contrib, meta, and sh_c, the rare copy-on-visible NEE value) stay indexed by
// path id for k_accumulate.
// ALT = false: pathTrace only (RayTracer::render's estimator; the other modes compile away).
// ALT = true: every per-pixel estimator of rtg_set_integrator, selected by a.mode.
// TAB = true: the scene's material and light records (at most RTG_LDS_MATS / RTG_LDS_LIGHTS) are
// copied into LDS while the payload and the hit triangle's shading record load, so the material a
// shading record names is an LDS read, not a dependent global fetch: the chain per path is payload ->
// shading record -> (texels of a texture larger than 1x1).
template <bool ALT, bool TAB>
__global__ __launch_bounds__(RTG_TB, RTG_SHADE_WAVES) void k_shade(SceneView s, ChunkArgs a, PathBufs p, int b) {
    __shared__ unsigned s_cnt[2][RTG_TB / 64];
    __shared__ unsigned s_base[2];
    __shared__ float4 s_sho[RTG_TB], s_shd[RTG_TB];  // NEE ray staged until its queue position is known
    __shared__ DevMat s_mat[TAB ? RTG_LDS_MATS : 1];
    __shared__ DevLight s_lt[TAB ? RTG_LDS_LIGHTS : 1];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const bool lean0 = b == 0;  // bounce 0: path id = position, camera origin, thr 1, PCG seed, canHitLight
    // This block's tile of 256 queue positions [base, base + 256), live below n: tile blockIdx / 8
    // of input segment blockIdx % 8 (Counters::ne8; bounce 0: the camera rays, positions = path
    // ids). Its continuing paths and NEE rays are appended to the same segment of the next queues:
    // a segment keeps its region of the image from bounce to bounce (it is k_trace's slice k, walked
    // by XCD k), and blocks running together append to 8 different counters.
    const unsigned cap = a.seg_tiles * RTG_TB;
    const unsigned sg = blockIdx.x & 7u;
    const unsigned base = sg * cap + (blockIdx.x >> 3) * RTG_TB;
    const unsigned n = sg * cap + p.ctr[b].ne8[32 * sg];
    if (base >= n) return;  // block-uniform
    // extension payload of this bounce (set b & 1, by queue position) and of the next (set (b+1) & 1)
    const float4* in_o = (b & 1) ? p.ray_o2 : p.ray_o;
    const float4* in_d = (b & 1) ? p.ray_d2 : p.ray_d;
    const float4* in_t = (b & 1) ? p.thr2 : p.thr;
    const unsigned long long* in_r = (b & 1) ? p.rng2 : p.rng;
    float4* out_o = (b & 1) ? p.ray_o : p.ray_o2;
    float4* out_d = (b & 1) ? p.ray_d : p.ray_d2;
    float4* out_t = (b & 1) ? p.thr : p.thr2;
    unsigned long long* out_r = (b & 1) ? p.rng : p.rng2;
    float4* contrib = p.contrib + (size_t)b * a.P;
    // material / light tables: global -> LDS directly (global_load_lds_dwordx4, no VGPRs), 16 B per
    // thread; a wave's lanes fill 64 consecutive pieces from the wave's base
    if (TAB) {
        typedef __attribute__((address_space(1))) const void* gptr_t;
        typedef __attribute__((address_space(3))) void* lptr_t;
        const unsigned w0 = threadIdx.x & ~63u;
        if ((int)threadIdx.x < 4 * s.n_mats)
            __builtin_amdgcn_global_load_lds((gptr_t)(reinterpret_cast<const float4*>(s.mats) + threadIdx.x),
                                             (lptr_t)(reinterpret_cast<float4*>(s_mat) + w0), 16, 0, 0);
        if ((int)threadIdx.x < 5 * s.n_lights)
            __builtin_amdgcn_global_load_lds((gptr_t)(reinterpret_cast<const float4*>(s.lights) + threadIdx.x),
                                             (lptr_t)(reinterpret_cast<float4*>(s_lt) + w0), 16, 0, 0);
    }
    // one 256-path tile per block: a finished block frees its slot for the next tile
    {
        const unsigned i = base + threadIdx.x;
        int pid = 0;
        bool want_ext = false, want_sh = false;
        // the next bounce's payload, written at its queue position once the block's compaction has
        // assigned it (the NEE shadow ray is written at once, by path id)
        float4 n_o = make_float4(0.0f, 0.0f, 0.0f, 0.0f), n_d = n_o, n_t = n_o;
        unsigned long long n_r = 0;
        const bool valid = i < n;
        // the payload and, on a hit, the triangle's shading record (issued before the tables' barrier)
        float4 ro = make_float4(a.cam.ox, a.cam.oy, a.cam.oz, 0.0f), rd = ro, h = ro;
        DevShade S;
        if (valid) {
            unsigned j = i;  // bounce 0: the pixel's camera ray and first hit (k_generate), shared by its samples
            if (lean0) {
                unsigned sl0;
                split_pid(a, i, j, sl0);
            }
            if (!lean0) ro = in_o[i];
            rd = in_d[j];
            h = p.hits[j];
            if (h.x < RTG_FLT_MAX) S = s.shade[__float_as_int(h.y)];
        }
        if (TAB) {
            // global_load_lds completes on vmcnt, not on the barrier: wait for it explicitly (the
            // payload loads above are then in too) before other waves read the tables.
            // tests/test_kernel_resources.py pins the s_waitcnt vmcnt(0) ahead of this s_barrier
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
        }
        if (valid) {
            pid = lean0 ? (int)i : __float_as_int(ro.w);  // the path id travels in ray_o.w
            const v3 o = mk(ro.x, ro.y, ro.z), d = mk(rd.x, rd.y, rd.z);
            const float4 thr4 = lean0 ? make_float4(1.0f, 1.0f, 1.0f, 0.0f) : in_t[i];
            v3 thr = mk(thr4.x, thr4.y, thr4.z);
            const int can_hit = lean0 ? 1 : (rd.w != 0.0f);  // canHitLight travels in ray_d.w
            unsigned lp, sl;
            split_pid(a, (unsigned)pid, lp, sl);
            const uint64_t inc = pcg_inc(a.pixlist[lp], a.s0 + sl);  // (carrying it in the payload: slower)
            uint64_t st = lean0 ? pcg_seed(a.seed, inc) : in_r[i];
            v3 c = mk(0.0f, 0.0f, 0.0f);
            int nterms = b + 1;
            // state carried past the environment lookup: a miss, or a path-traced hit (stage 1:
            // its light sample taken, its shading, shadow ray and BSDF sample to come)
            bool miss = false, env_need = false, env_light = false, spec = false;
            int stage = 0, mid = 0;
            v3 env_dir = d, x = o, sn = d, alb = d, l_p2 = o, l_em = d;
            float l_g = 0.0f, l_pdf = 0.0f;
            if (ALT && a.mode == RTG_INTEGRATOR_DIRECT_MIS && b == 1) {
                // computeDirectMIS, second half (Renderer.h:520-553): the BSDF-sampled ray's hit.
                // thr = (bsdf value, bsdf pdf); scratch planes 2/3 = (x, light pdf * pmf) and
                // (max(0, wi.sN), env-sample flag); contrib plane 0 .w = 1 iff an env NEE sample was
                // visible, in which case the reference has already returned (:508-516).
                const float4 A = p.contrib[(size_t)2 * a.P + pid], B = p.contrib[(size_t)3 * a.P + pid];
                const float4 c0 = p.contrib[pid];
                c = mk(0.0f, 0.0f, 0.0f);
                if (B.y != 0.0f && c0.w == 1.0f) {
                    nterms = 1;
                } else if (h.x < RTG_FLT_MAX) {
                    const DevMat& M = TAB ? s_mat[__float_as_int(S.d.w)] : s.mats[__float_as_int(S.d.w)];
                    if (M.is_light) {
                        const float alpha = h.z, beta = h.w, gamma = 1.0f - (alpha + beta);
                        const v3 x2 = add(o, muls(d, h.x));
                        const v3 n0 = mk(S.a.x, S.a.y, S.a.z), n1 = mk(S.a.w, S.b.x, S.b.y), n2 = mk(S.b.z, S.b.w, S.c.x);
                        v3 sn2 = normalize(add(add(muls(n0, alpha), muls(n1, beta)), muls(n2, gamma)));
                        if (M.two_sided && dot(neg(d), sn2) < 0) sn2 = neg(sn2);
                        v3 wi = sub(x2, mk(A.x, A.y, A.z));
                        const float dist2 = length_sq(wi);
                        wi = normalize(wi);
                        const float cos_l = wmax(0.0f, dot(neg(wi), sn2));
                        const float pls = pdf_area_to_solid(A.w, dist2, cos_l);
                        const float wgt = balance_heuristic(thr4.w, pls);
                        c = divs(muls(muls(mul(thr, mk(M.emission.x, M.emission.y, M.emission.z)), B.x), wgt), thr4.w);
                    }
                }
            } else if (!(h.x < RTG_FLT_MAX)) {
                // miss: background->evaluate(r.dir), not weighted by throughput (Renderer.h:390);
                // direct() and viewNormals() return black. BackgroundColour(0) is black; an
                // environment map is evaluated below, at the lane's one environment lookup.
                env_need = (!ALT || a.mode == RTG_INTEGRATOR_PATH || a.mode == RTG_INTEGRATOR_ALBEDO) && s.env_tex >= 0;
                miss = true;
            } else {
                const float alpha = h.z, beta = h.w, gamma = 1.0f - (alpha + beta);
                const float t = h.x;
                x = add(o, muls(d, t));  // Ray::at
                mid = __float_as_int(S.d.w);
                const DevMat& M = TAB ? s_mat[mid] : s.mats[mid];
                const v3 n0 = mk(S.a.x, S.a.y, S.a.z), n1 = mk(S.a.w, S.b.x, S.b.y), n2 = mk(S.b.z, S.b.w, S.c.x);
                sn = normalize(add(add(muls(n0, alpha), muls(n1, beta)), muls(n2, gamma)));
                const float tu = (S.c.y * alpha + S.c.w * beta) + S.d.y * gamma;
                const float tv = (S.c.z * alpha + S.d.x * beta) + S.d.z * gamma;
                const v3 wo = neg(d);
                if (M.two_sided && dot(wo, sn) < 0) sn = neg(sn);
                if (ALT && a.mode == RTG_INTEGRATOR_NORMALS) {  // viewNormals (Renderer.h:572-582)
                    c = mk(fabsf(sn.x), fabsf(sn.y), fabsf(sn.z));
                } else if (M.is_light) {
                    c = (ALT && a.mode != RTG_INTEGRATOR_PATH) ? mk(M.emission.x, M.emission.y, M.emission.z)  // emit()
                        : can_hit ? mul(thr, mk(M.emission.x, M.emission.y, M.emission.z)) : mk(0.0f, 0.0f, 0.0f);
                } else if (ALT && a.mode == RTG_INTEGRATOR_ALBEDO) {  // BSDF::evaluate(sd, (0,1,0))
                    const v3 alb = tex_sample(s, M, tu, tv);
                    c = M.kind == RTG_MAT_MIRROR ? alb : (M.kind == RTG_MAT_GLASS ? mk(0.0f, 0.0f, 0.0f) : divs_pi(alb));
                } else if (ALT && a.mode == RTG_INTEGRATOR_DIRECT_MIS) {
                    // computeDirectMIS, first half (Renderer.h:474-519): one light sample weighted by
                    // the balance heuristic (its shadow ray), then one BSDF sample (its extension ray)
                    const frame fr = frame_from(sn);
                    c = mk(0.0f, 0.0f, 0.0f);
                    if (!(M.kind == RTG_MAT_MIRROR || M.kind == RTG_MAT_GLASS)) {
                        const int nl = s.n_lights;
                        const float pmf = s.pmf;  // 1.f / (float)nl
                        int li = (int)((float)nl * pcg_next(st, inc));
                        li = (nl - 1) < li ? (nl - 1) : li;
                        const DevLight L = TAB ? s_lt[li] : s.lights[li];
                        const v3 f = divs_pi(tex_sample(s, M, tu, tv));  // BSDF::evaluate
                        float pdf;
                        float env_flag = 0.0f;
                        if (__float_as_int(L.v1t.w) == 0) {
                            const float r1 = pcg_next(st, inc);
                            const float r2 = pcg_next(st, inc);
                            const float la = 1 - sqrtf(r1);
                            const float lb = r2 * sqrtf(r1);
                            const float lg = 1.0f - (la + lb);
                            pdf = L.v2.w;  // 1.0f / area
                            const v3 p2 = add(add(muls(mk(L.v0a.x, L.v0a.y, L.v0a.z), la), muls(mk(L.v1t.x, L.v1t.y, L.v1t.z), lb)),
                                              muls(mk(L.v2.x, L.v2.y, L.v2.z), lg));
                            v3 wi = sub(p2, x);
                            const float l2 = length_sq(wi);
                            wi = normalize(wi);
                            const float cos_s = wmax(dot(wi, sn), 0.0f);
                            const float cos_l = wmax(-dot(wi, mk(L.gn.x, L.gn.y, L.gn.z)), 0.0f);
                            const float g = (cos_s * cos_l) / l2;
                            if (g > 0) {
                                const float pdf_b = bsdf_pdf_lambert(fr, wi);
                                const float pls = pdf_area_to_solid(pdf * pmf, l2, cos_l);
                                const float wgt = balance_heuristic(pls, pdf_b);
                                const v3 r = add(mk(0.0f, 0.0f, 0.0f),
                                                 divs(muls(muls(mul(f, mk(L.em.x, L.em.y, L.em.z)), g), wgt), pmf * pdf));
                                v3 sd = sub(p2, x);
                                const float maxt = sqrtf(length_sq(sd)) - (2.0f * RTG_EPS);
                                sd = normalize(sd);
                                const v3 so = add(x, muls(sd, RTG_EPS));
                                s_sho[threadIdx.x] = make_float4(so.x, so.y, so.z, maxt);
                                s_shd[threadIdx.x] = make_float4(sd.x, sd.y, sd.z, 1.0f);  // copy sh_c if visible
                                p.sh_c[pid] = make_float4(r.x, r.y, r.z, 0.0f);
                                want_sh = true;
                            }
                        } else {
                            const float q2 = pcg_next(st, inc);
                            const float q1 = pcg_next(st, inc);
                            const v3 wi = uniform_sample_sphere(q1, q2);
                            pdf = uniform_sphere_pdf();
                            const float g = wmax(dot(wi, sn), 0.0f);
                            if (g > 0) {
                                const v3 r = divs(muls(mul(f, env_eval(s, wi)), g), pmf * pdf);
                                const v3 p2 = add(x, muls(wi, 10000.0f));
                                v3 sd = sub(p2, x);
                                const float maxt = sqrtf(length_sq(sd)) - (2.0f * RTG_EPS);
                                sd = normalize(sd);
                                const v3 so = add(x, muls(sd, RTG_EPS));
                                s_sho[threadIdx.x] = make_float4(so.x, so.y, so.z, maxt);
                                s_shd[threadIdx.x] = make_float4(sd.x, sd.y, sd.z, 1.0f);  // copy sh_c if visible
                                p.sh_c[pid] = make_float4(r.x, r.y, r.z, 1.0f);  // .w: env sample visible
                                want_sh = true;
                                env_flag = 1.0f;
                            }
                        }
                        // BSDF sample and its ray (Renderer.h:520-525)
                        v3 val;
                        float pdf_b;
                        PcgSampler smp{st, inc};
                        const v3 wib = bsdf_sample(M.kind, M.int_ior, M.ext_ior, tex_sample(s, M, tu, tv), fr, wo, smp,
                                                   val, pdf_b);
                        st = smp.s;
                        const v3 no = add(x, muls(wib, RTG_EPS));
                        n_o = make_float4(no.x, no.y, no.z, __int_as_float(pid));
                        n_d = make_float4(wib.x, wib.y, wib.z, 0.0f);
                        n_t = make_float4(val.x, val.y, val.z, pdf_b);
                        n_r = st;
                        p.contrib[(size_t)2 * a.P + pid] = make_float4(x.x, x.y, x.z, pdf * pmf);
                        p.contrib[(size_t)3 * a.P + pid] = make_float4(wmax(0.0f, dot(wib, sn)), env_flag, 0.0f, 0.0f);
                        want_ext = true;
                        nterms = 2;
                    }
                } else {
                    // computeDirect's light sample (Renderer.h:423-447); its shading, shadow ray and
                    // the BSDF sample follow the lane's environment lookup below
                    spec = M.kind == RTG_MAT_MIRROR || M.kind == RTG_MAT_GLASS;
                    // albedo->sample(tu, tv): one fetch for BSDF::evaluate (NEE) and BSDF::sample
                    alb = tex_sample(s, M, tu, tv);
                    if (!spec) {
                        const int nl = s.n_lights;
                        int li = (int)((float)nl * pcg_next(st, inc));
                        li = (nl - 1) < li ? (nl - 1) : li;  // (std::min)(a, b)
                        const DevLight L = TAB ? s_lt[li] : s.lights[li];
                        if (__float_as_int(L.v1t.w) == 0) {  // AreaLight::sample -> Triangle::sample
                            const float r1 = pcg_next(st, inc);
                            const float r2 = pcg_next(st, inc);
                            const float la = 1 - sqrtf(r1);
                            const float lb = r2 * sqrtf(r1);
                            const float lg = 1.0f - (la + lb);
                            l_pdf = L.v2.w;  // 1.0f / area
                            l_p2 = add(add(muls(mk(L.v0a.x, L.v0a.y, L.v0a.z), la), muls(mk(L.v1t.x, L.v1t.y, L.v1t.z), lb)),
                                       muls(mk(L.v2.x, L.v2.y, L.v2.z), lg));
                            l_em = mk(L.em.x, L.em.y, L.em.z);
                            v3 wi = sub(l_p2, x);
                            const float l2 = length_sq(wi);
                            wi = normalize(wi);
                            l_g = (wmax(dot(wi, sn), 0.0f) * wmax(-dot(wi, mk(L.gn.x, L.gn.y, L.gn.z)), 0.0f)) / l2;
                        } else {  // EnvironmentMap::sample: uniformSampleSphere(next(), next())
                            const float q2 = pcg_next(st, inc);  // evaluated first -> r2
                            const float q1 = pcg_next(st, inc);  // -> r1
                            const v3 wi = uniform_sample_sphere(q1, q2);
                            l_pdf = uniform_sphere_pdf();
                            l_g = wmax(dot(wi, sn), 0.0f);
                            l_p2 = add(x, muls(wi, 10000.0f));
                            env_dir = wi;  // its radiance: EnvironmentMap::evaluate(wi), below (used iff g > 0)
                            env_need = l_g > 0;
                            env_light = true;
                        }
                    }
                    stage = 1;
                }
            }
            // The lane's one environment lookup: a miss's background and an environment light
            // sample's radiance are the same EnvironmentMap::evaluate (Lights.h:150-157), so a wave
            // holding both kinds of lane runs it once instead of in two divergent branches.
            const v3 E = env_need ? env_eval(s, env_dir) : mk(0.0f, 0.0f, 0.0f);
            if (miss) c = E;
            if (stage == 1) {
                const DevMat& M = TAB ? s_mat[mid] : s.mats[mid];
                const v3 wo = neg(d);
                const frame fr = frame_from(sn);
                // ---- computeDirect (Renderer.h:423-473), after the light sample above
                v3 ld = mk(0.0f, 0.0f, 0.0f);
                bool ld_pre = false;  // contrib takes the visible NEE value now
                v3 cpre = ld;
                if (!spec && l_g > 0) {
                    const float pmf = s.pmf;  // 1.f / (float)nl
                    const v3 emitted = env_light ? E : l_em;
                    // Scene::visible(x, p2)
                    v3 sd = sub(l_p2, x);
                    const float maxt = sqrtf(length_sq(sd)) - (2.0f * RTG_EPS);
                    sd = normalize(sd);
                    const v3 so = add(x, muls(sd, RTG_EPS));
                    const v3 f = divs_pi(alb);  // BSDF::evaluate
                    ld = divs(muls(mul(f, emitted), l_g), pmf * l_pdf);
                    const v3 cvis = mul(thr, ld);
                    s_sho[threadIdx.x] = make_float4(so.x, so.y, so.z, maxt);
                    // Visible is the common case: contrib takes thr * Ld now and k_trace
                    // writes thr * 0 = +0 on occlusion. When thr * 0 is not +0 (a non-finite
                    // throughput) the value goes through sh_c and is copied on visibility.
                    const v3 z = mul(thr, mk(0.0f, 0.0f, 0.0f));
                    const bool plain = (__float_as_uint(z.x) | __float_as_uint(z.y) | __float_as_uint(z.z)) == 0u;
                    s_shd[threadIdx.x] = make_float4(sd.x, sd.y, sd.z, plain ? 0.0f : 1.0f);
                    if (!plain) p.sh_c[pid] = make_float4(cvis.x, cvis.y, cvis.z, 0.0f);
                    ld_pre = plain;
                    cpre = cvis;
                    want_sh = true;
                }
                // direct = thr * Ld, with Ld = 0 until the shadow ray says visible
                c = ld_pre ? cpre : mul(thr, mk(0.0f, 0.0f, 0.0f));
                if ((!ALT || a.mode == RTG_INTEGRATOR_PATH) && b <= a.max_depth) {
                    const float rrp = wmin(lum(thr), 0.9f);
                    if (pcg_next(st, inc) < rrp) {
                        thr = divs(thr, rrp);
                        // ---- BSDF::sample
                        v3 ind;
                        float pdf;
                        PcgSampler smp{st, inc};
                        const v3 wi = bsdf_sample(M.kind, M.int_ior, M.ext_ior, alb, fr, wo,
                                                  smp, ind, pdf);
                        st = smp.s;
                        if (spec) thr = divs(mul(thr, ind), pdf);
                        else thr = divs(muls(mul(thr, ind), fabsf(dot(wi, sn))), pdf);
                        const v3 no = add(x, muls(wi, RTG_EPS));
                        n_o = make_float4(no.x, no.y, no.z, __int_as_float(pid));
                        n_d = make_float4(wi.x, wi.y, wi.z, spec ? 1.0f : 0.0f);  // canHitLight
                        want_ext = true;
                        n_t = make_float4(thr.x, thr.y, thr.z, 0.0f);
                        n_r = st;
                        nterms = (b + 1) | ((spec ? 1 : 0) << 8);
                    }
                }
            }
            contrib[pid] = make_float4(c.x, c.y, c.z, 0.0f);
            p.meta[pid] = nterms;
        }
        // ---- block-level compaction of path ids into the next queues (one atomic per queue)
        const unsigned long long me = __ballot(want_ext);
        const unsigned long long ms = __ballot(want_sh);
        if (lane == 0) {
            s_cnt[0][wave] = (unsigned)__popcll(me);
            s_cnt[1][wave] = (unsigned)__popcll(ms);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned te = 0, ts = 0;
            for (int w = 0; w < RTG_TB / 64; ++w) {
                te += s_cnt[0][w];
                ts += s_cnt[1][w];
            }
            // (at most seg_tiles blocks append to a segment: it cannot overflow)
            s_base[0] = te ? atomicAdd(&p.ctr[b + 1].ne8[32 * sg], te) + sg * cap : 0u;
            s_base[1] = ts ? atomicAdd(&p.ctr[b].ns8[32 * sg], ts) + sg * cap : 0u;
        }
        __syncthreads();
        unsigned oe = s_base[0], os = s_base[1];
        for (int w = 0; w < wave; ++w) {
            oe += s_cnt[0][w];
            os += s_cnt[1][w];
        }
        if (want_ext) {
            const unsigned j = oe + prefix_lt(me);
            out_o[j] = n_o;
            out_d[j] = n_d;
            out_t[j] = n_t;
            out_r[j] = n_r;
        }
        if (want_sh) {
            const unsigned j = os + prefix_lt(ms);
            p.shq[j] = (unsigned)pid;  // k_trace writes the path's contrib entry on occlusion
            p.sh_o[j] = s_sho[threadIdx.x];
            p.sh_d[j] = s_shd[threadIdx.x];
        }
        __syncthreads();
    }
}


// The launch of one shading bounce (render_impl): the pathTrace-only kernel or the one holding every
// per-pixel estimator, with or without the LDS material / light tables.
int launch_shade(bool alt, bool tab, unsigned grid, hipStream_t st, const SceneView& s, const ChunkArgs& a,
                 const PathBufs& p, int b) {
    auto kern = alt ? (tab ? k_shade<true, true> : k_shade<true, false>)
                    : (tab ? k_shade<false, true> : k_shade<false, false>);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(RTG_TB), 0, st, s, a, p, b);
    LAUNCH_OK("k_shade");
    return RTG_OK;
}
