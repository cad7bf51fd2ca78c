// rtg_kernels.hip — MI355X (gfx950) wavefront path tracer: kernels + the C-ABI of include/rtg.h.
//
// One RayTracer::render() (RTBase/Renderer.h:876) = one sample for every pixel. Here a "chunk" is
// ns samples x npix pixels = P paths in flight, advanced bounce by bounce:
//
//   k_generate        Camera::generateRay (Scene.h:43-54) at pixel centres, PCG32 seed, path state
//   for b in 0 .. max_depth+2:                                   (pathTrace recursion, depth = b)
//     k_shade (b > 0)  bounce b-1: calculateShadingData + emission + computeDirect (NEE sample,
//                      shadow ray) + Russian roulette + BSDF::sample + throughput
//                      (Renderer.h:328-392, 423-473) -> compacts continuing paths into the next
//                      extension queue and NEE rays into the shadow queue (one atomic per block)
//     k_trace          one launch for both ray kinds: Scene::traverse (Scene.h:107-130,
//                      Geometry.h:399-434) for the extension rays of bounce b and Scene::visible
//                      (Scene.h:161-169, Geometry.h:435-462) for the shadow rays of bounce b-1
//   k_accumulate      right-nested radiance sum d0 + (d1 + (... + dk)) (Renderer.h:388) per path,
//                      then film += L in sample order (Film::splat, Imaging.h:209-232)
//
// Exactness: each path's result is independent of queue order and of traversal order. Closest hit
// returns the (t, triangle index) lexicographic minimum over the reference's reachable triangles,
// which is what the reference's left-first DFS with strict '<' keeps; box tests use the reference's
// exact slab arithmetic, and distance culling only removes boxes whose conservatively inflated entry
// is beyond the current hit.
#include "rtg_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

// ------------------------------------------------------------------ traversal
// Persistent lanes with per-lane ray replacement: a wave takes 64 ray indices at a time from the
// queue (one atomic per 64 rays) into a wave-uniform pool, and every lane whose ray terminates
// immediately takes the next index from the pool. Without replacement a wave runs until its
// longest ray finishes (measured SIMD efficiency ~27 %).
// Work slice k of a trace launch. Path tracer (segmented queues, io.seg_cap != 0; io.fetch8: one
// counter per slice, by blockIdx % 8, i.e. one per XCD): slice k is queue segment k, its extension
// rays at positions [k * seg_cap, + elen) and then its shadow rays at the same shadow positions, so
// every XCD walks long closest-hit rays first and ends on any-hit rays; len rays in all. Otherwise
// (one counter: light tracer, ray queries): every ray, extension rays first.
static __device__ __forceinline__ void trace_slice(const TraceIO& io, unsigned nc, unsigned n, int k, unsigned& elo,
                                                   unsigned& elen, unsigned& len) {
    if (io.seg_cap) {
        elo = (unsigned)k * io.seg_cap;
        elen = io.seg_ne ? io.seg_ne[32 * k] : 0u;
        len = elen + (io.seg_ns ? io.seg_ns[32 * k] : 0u);
    } else {
        elo = 0;
        elen = nc;
        len = n;
    }
}

// SMALL: the scene's wide nodes, triangle records and leaf boxes are copied into LDS at the start of
// each block (SceneView::img, small scenes only) and the walk reads them there; the LDS stack is then
// RTG_STACK_SMALL entries, so the block's LDS stays below 5 KB (7 one-wave blocks per SIMD, as the
// global walk's 16-entry stack).
template <bool COUNT, bool SMALL>
__global__ __launch_bounds__(RTG_TTB) __attribute__((amdgpu_waves_per_eu(RTG_TRACE_WPE)))
void k_trace(SceneView s, TraceIO io) {
    constexpr int STK = SMALL ? RTG_STACK_SMALL : RTG_STACK;
    __shared__ int stk[STK][RTG_TTB];
    __shared__ float kstk[COUNT ? STK : 1][RTG_TTB];  // COUNT only: entry key of each push
    __shared__ float4 s_img[SMALL ? RTG_SMALL_F4 : 1];
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const unsigned gthreads = gridDim.x * blockDim.x;
    const unsigned gtid = blockIdx.x * blockDim.x + tid;
    // extension index span: the ray count, or (segmented queues) all 8 segments' positions
    const unsigned nc = io.seg_cap ? 8u * io.seg_cap : (io.count ? *io.count : 0u);
    const unsigned n = nc + (io.scount ? *io.scount : 0u);
    unsigned long long c_nodes = 0, c_tris = 0, c_snodes = 0, c_stris = 0, c_slots = 0, c_nstep = 0, c_lstep = 0,
                       c_cullpop = 0, c_pops = 0, c_lslots = 0, c_lbox = 0;
    unsigned c_tails = 0;  // triangle records whose last 16 B were fetched (COUNT)
    // COUNT: why a lane is not stepping a node in an iteration: no ray, its walk done but its parked
    // leaf not run yet, a leaf reached while both parked-leaf slots are full, retiring this iteration, a leaf
    // popped last iteration (parked in this one)
    unsigned long long c_idle_e = 0, c_idle_ll = 0, c_idle_lb = 0, c_idle_r = 0, c_idle_lp = 0;
    unsigned pool_base = 0, pool_left = 0, last_b = 0;  // wave-uniform
    const unsigned tail_rays = (gthreads / 64u) * (unsigned)RTG_FETCH * RTG_FETCH_TAIL / (io.fetch8 ? 8u : 1u);
    // the 8 slices (trace_slice) in LDS, read when a wave fetches work: the loop keeps only the
    // slice number in a register
    __shared__ unsigned s_tab[3][8];
    if (tid < 8) {
        unsigned elo, elen, len;
        trace_slice(io, nc, n, tid, elo, elen, len);
        s_tab[0][tid] = elo;
        s_tab[1][tid] = elen;
        s_tab[2][tid] = len;
        // the host's next k_shade grid (TraceIO::hcnt): a volatile vector store, emitted with the
        // system-scope bits (sc0 sc1). (__hip_atomic_store at system scope cost the walk 4 VGPR spills)
        if (io.hcnt && blockIdx.x == 0) ((volatile unsigned*)io.hcnt)[tid] = elen;
    }
    if (SMALL)
        for (int i = tid; i < s.img_n4; i += RTG_TTB) s_img[i] = s.img[i];
    __syncthreads();
    const DevTri48* tris = SMALL ? reinterpret_cast<const DevTri48*>(s_img + s.img_tri) : s.tris48;
    const float4* lboxes = (SMALL && RTG_SMALL_LB) ? s_img + s.img_lb : s.leafbox;
    int slice = io.fetch8 ? (int)(blockIdx.x & 7u) : 0, tried = 0;  // wave-uniform
    unsigned s_len = __builtin_amdgcn_readfirstlane(s_tab[2][slice]);
    bool drained = false;                   // wave-uniform
    bool have = false;
    unsigned ri = 0;
    v3 o = mk(0, 0, 0), d = mk(0, 0, 0), inv = mk(0, 0, 0);
    float tbest = 0.0f, omag = 0.0f, dmag = 0.0f, delta = 0.0f, bu = 0.0f, bv = 0.0f;
    int bid = -1, pid = 0, cur = RTG_EXIT, sp = 0, pend = RTG_EXIT;
    int pend2 = RTG_EXIT;  // RTG_PEND2: a second parked leaf (the leaf phase runs pend, then pend2 moves up)
    bool occluded = false, wide = false, anyr = false;  // anyr: this lane's ray is a shadow ray
    const unsigned wslot = gtid >> 6;
    // RTG_DEBUG capture: the ray's record fetches in order (cap_k of them so far)
    unsigned cap_ri = 0, cap_k = 0;
    uint4 cap_q = make_uint4(0, 0, 0, 0);
    auto capture = [&](unsigned type, unsigned idx) {
        if (!RTG_DEBUG || !io.cap) return;
        if (cap_k < RTG_CAP_LEN) {
            const unsigned e = (type << 30) | idx;
            const unsigned j = cap_k & 3;
            cap_q.x = j == 0 ? e : cap_q.x;
            cap_q.y = j == 1 ? e : cap_q.y;
            cap_q.z = j == 2 ? e : cap_q.z;
            cap_q.w = j == 3 ? e : cap_q.w;
            if (j == 3) io.cap[(size_t)(cap_k >> 2) * io.cap_n + cap_ri] = cap_q;
        }
        ++cap_k;
    };
    if (RTG_DEBUG && io.wtime && lane == 0) io.wtime[3 * wslot] = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        // ---- retire finished rays
        if (have && cur == RTG_EXIT && pend == RTG_EXIT && (!RTG_PEND2 || pend2 == RTG_EXIT)) {
            if (anyr) {
                if (io.visible) io.visible[pid] = occluded ? 0 : 1;
                else if (bid == -2 ? occluded : !occluded)
                    io.contrib[pid] = bid == -2 ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : io.sray_c[pid];
            } else {
                io.hits[pid] = make_float4(tbest, __int_as_float(bid), bu, bv);
            }
            if (RTG_DEBUG && io.cap) {
                const unsigned k = min(cap_k, (unsigned)RTG_CAP_LEN);
                if (k & 3) io.cap[(size_t)(k >> 2) * io.cap_n + cap_ri] = cap_q;
                io.cap_len[cap_ri] = cap_k;  // the true count; the first RTG_CAP_LEN are kept
            }
            have = false;
        }
        // ---- refill idle lanes from the wave's pool
        const unsigned long long im = __ballot(!have);
        if (im != 0 && !drained && (__popcll(im) >= RTG_REFILL || __ballot(have) == 0)) {
            // wave-uniform fetch: big batches (one atomic per fetch_big rays) until about
            // RTG_FETCH_TAIL rounds of them are left in the slice, judged from this wave's previous
            // fetch, then 64 (shorter drain tails). With io.fetch8 the index space is cut into 8
            // slices with a counter each (the atomics of one counter serialise); a wave starts on
            // slice blockIdx % 8 and moves on to the next slice when its own runs dry.
            while (pool_left == 0) {
                const bool tail = last_b + tail_rays >= s_len;
                const unsigned g = tail ? (unsigned)RTG_TAIL_BATCH : (unsigned)RTG_FETCH;
                unsigned b = 0;
                if (lane == 0) b = atomicAdd(io.fetch8 ? io.fetch8 + 32 * slice : io.fetch, g);
                b = __builtin_amdgcn_readfirstlane(b);  // wave-uniform: keeps the fetch state in SGPRs
                last_b = b;
                if (b < s_len) {
                    pool_base = b;
                    pool_left = min(g, s_len - b);
                } else if (!io.fetch8 || ++tried == 8) {
                    drained = true;
                    if (RTG_DEBUG && io.wtime && lane == 0) io.wtime[3 * wslot + 1] = __builtin_amdgcn_s_memrealtime();
                    break;
                } else {
                    slice = (slice + 1) & 7;
                    s_len = __builtin_amdgcn_readfirstlane(s_tab[2][slice]);
                    last_b = s_len;  // a stolen slice is near its end: small batches
                }
            }
            if (pool_left > 0) {
                const unsigned pos = prefix_lt(im);
                const unsigned take = min((unsigned)__popcll(im), pool_left);
                if (!have && pos < take) {
                    const unsigned j = pool_base + pos;  // index within the slice
                    const unsigned s_elo = s_tab[0][slice], s_elen = s_tab[1][slice];
                    ri = j < s_elen ? s_elo + j : nc + s_elo + (j - s_elen);
                    have = true;
                    if (RTG_DEBUG) { cap_ri = ri; cap_k = 0; }
                    anyr = ri >= nc;
                    pid = (int)(anyr ? io.squeue[ri - nc] : (io.queue ? io.queue[ri] : ri));
                    // io.spos: the shadow ray sits at its shadow-queue position (no dependence on the
                    // id load; the id is needed when the ray retires)
                    const unsigned sk = io.spos ? ri - nc : (unsigned)pid;
                    const float4 ro = anyr ? io.sray_o[sk] : (io.ray_o ? io.ray_o[pid] : io.cam_o);
                    const float4 rd = anyr ? io.sray_d[sk] : io.ray_d[pid];
                    // sh_d.w != 0: the shadow value is in sray_c and is copied on visibility;
                    // 0: k_shade already stored it in contrib, which is cleared on occlusion
                    // (kept in bid, which a shadow ray does not use: -2 = value already in contrib)
                    o = mk(ro.x, ro.y, ro.z);
                    d = mk(rd.x, rd.y, rd.z);
                    tbest = anyr ? ro.w : RTG_FLT_MAX;
                    inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);  // Ray::init
                    omag = s.cull_scale + fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
                    dmag = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
                    delta = RTG_CULL_REL * (omag + (tbest < RTG_FLT_MAX ? tbest * dmag : 0.0f));
                    bid = (anyr && !io.visible && rd.w == 0.0f) ? -2 : -1;
                    bu = bv = 0.0f;
                    occluded = false;
                    sp = 0;
                    pend = RTG_EXIT;
                    pend2 = RTG_EXIT;
                    // Wide walk only when every 1/d component is finite and nonzero (no NaN slab
                    // terms): then a passing descendant box implies its skipped ancestors pass.
                    // (|1/d| <= 2^64 and scene scale in [2^-60, 2^60] keep every product of the
                    // compressed walk finite and normal.)
                    wide = io.wide && s.usew && fabsf(inv.x) <= 0x1p64f && fabsf(inv.y) <= 0x1p64f &&
                           fabsf(inv.z) <= 0x1p64f && inv.x != 0.0f && inv.y != 0.0f && inv.z != 0.0f;
                    const float* rb = s.root_box;
                    cur = slab_exact(rb[0], rb[1], rb[2], rb[3], rb[4], rb[5], o, inv)
                              ? (wide ? s.root_wordw : s.root_word) : RTG_EXIT;
                }
                pool_base += take;
                pool_left -= take;
            }
        }
        if (drained && __ballot(have) == 0) break;
        if (COUNT) {
            c_slots += 64;
            c_nstep += (have && cur >= 0) ? 1 : 0;
            c_idle_e += !have ? 1 : 0;
            c_idle_ll += (have && cur == RTG_EXIT && pend != RTG_EXIT) ? 1 : 0;
            c_idle_lb += (have && cur < 0 && cur != RTG_EXIT && pend != RTG_EXIT && (!RTG_PEND2 || pend2 != RTG_EXIT)) ? 1 : 0;
            c_idle_r += (have && cur == RTG_EXIT && pend == RTG_EXIT) ? 1 : 0;
            c_idle_lp += (have && cur < 0 && cur != RTG_EXIT && (pend == RTG_EXIT || (RTG_PEND2 && pend2 == RTG_EXIT))) ? 1 : 0;
        }
        if (!have || (cur == RTG_EXIT && pend == RTG_EXIT && (!RTG_PEND2 || pend2 == RTG_EXIT))) continue;
        // Leaf: the reference's leaf loop (Geometry.h:420-431 / 446-458) over 1-2 triangles (a wide
        // leaf slot may join sibling reference leaves: up to RTG_LEAF_SPAN triangles).
        auto leaf = [&](const int word) {
            const int code = ~word;
            const int start = code / RTG_LEAF_SPAN;  // leaf word ~(start * RTG_LEAF_SPAN + count - 1)
            const int cnt = (code % RTG_LEAF_SPAN) + 1;
            for (int k = 0; k < cnt; ++k) {
                const int tri = start + k;
                if (COUNT) (anyr ? c_stris : c_tris) += 1;
                capture(1u, (unsigned)tri);
                float t, u, v;
                const bool hit = tri_intersect48p(tris + tri, o, d, [&](float tt) {
                    return anyr ? (tt < tbest && tt > RTG_EPS) : (tt <= tbest && tt > RTG_EPS);
                }, t, u, v, c_tails);
                if (hit) {
                    bool cand = anyr ? !(t >= tbest || t <= RTG_EPS)
                                     : (t > RTG_EPS && (t < tbest || (t == tbest && tri < bid)));
                    if (cand && wide) {
                        // the exact box of the reference leaf holding this triangle (stored per
                        // triangle: a wide leaf slot may join sibling reference leaves)
                        const float4 b0 = lboxes[2 * tri], b1 = lboxes[2 * tri + 1];
                        if (COUNT) c_lbox += 1;
                        capture(2u, (unsigned)tri);
                        cand = slab_exact(b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, o, inv);
                    }
                    if (!cand) {
                    } else if (anyr) {
                        occluded = true;
                    } else {
                        tbest = t;
                        bid = tri;
                        bu = u;
                        bv = v;
                        delta = RTG_CULL_REL * (omag + tbest * dmag);
                    }
                }
            }
        };
        // ---- one traversal step
        if (cur >= 0 && wide) {
            int wd[4];
            float key[4];
            {
                capture(0u, (unsigned)cur);
                const float4* np = SMALL ? s_img + 4 * cur : s.nodesq[cur].q;
                const float4 h0 = np[0], h1 = np[1], h2 = np[2], h3 = np[3];
                const unsigned ex = __float_as_uint(h0.w);
                const float sx = __uint_as_float((ex & 255u) << 23);
                const float sy = __uint_as_float(((ex >> 8) & 255u) << 23);
                const float sz = __uint_as_float(((ex >> 16) & 255u) << 23);
                const unsigned p0 = __float_as_uint(h1.x), p1 = __float_as_uint(h1.y), p2 = __float_as_uint(h1.z);
                const unsigned p3 = __float_as_uint(h1.w), p4 = __float_as_uint(h2.x), p5 = __float_as_uint(h2.y);
                wd[0] = __float_as_int(h2.z);
                wd[1] = __float_as_int(h2.w);
                wd[2] = __float_as_int(h3.x);
                wd[3] = __float_as_int(h3.y);
                // Conservative slot test in ray-relative form. Exactness does not need the exact slab
                // test here: a candidate hit is accepted only after its reference leaf box passes the
                // exact test, so a slot test only has to pass whenever the exact test on a reference
                // box inside the slot passes. Per axis, with s the power-of-two step:
                //   near entry  tn = fma(q_near, s*inv, ((origin + mn) - o) * inv)
                //   far exit    tf = fma(q_far,  s*inv, ((origin - mn) - o) * inv)
                // mn moves the near plane (and -mn the far plane) outward by mu = 2^-16 (scale + |o|).
                // The rounding of this form plus the reference's own is below 2^-19.5 (scale + |o|)|inv|
                // per plane, inside the mu |inv| margin, so tn <= the reference entry
                // and tf >= the reference exit of every box the slot contains.
                // Cull key: max(tn) - (delta - mu) * max|inv| is below the entry of the slot's box
                // inflated by delta (slab_cull_entry's conservative bound).
                const bool px = inv.x > 0.0f, py = inv.y > 0.0f, pz = inv.z > 0.0f;
                const unsigned nqx = px ? p0 : p3, fqx = px ? p3 : p0;
                const unsigned nqy = py ? p1 : p4, fqy = py ? p4 : p1;
                const unsigned nqz = pz ? p2 : p5, fqz = pz ? p5 : p2;
                const float mu = RTG_CULL_REL * omag;
                const float mnx = px ? -mu : mu, mny = py ? -mu : mu, mnz = pz ? -mu : mu;
                // packed FP32 (v_pk_*): per-component IEEE results identical to the scalar ops
                const f2 ax2 = ((f2){h0.x, h0.x} + (f2){mnx, -mnx} - (f2){o.x, o.x}) * (f2){inv.x, inv.x};
                const f2 ay2 = ((f2){h0.y, h0.y} + (f2){mny, -mny} - (f2){o.y, o.y}) * (f2){inv.y, inv.y};
                const f2 az2 = ((f2){h0.z, h0.z} + (f2){mnz, -mnz} - (f2){o.z, o.z}) * (f2){inv.z, inv.z};
                const float six = sx * inv.x, siy = sy * inv.y, siz = sz * inv.z;
                const f2 six2 = {six, six}, siy2 = {siy, siy}, siz2 = {siz, siz};
                const f2 anx2 = {ax2.x, ax2.x}, afx2 = {ax2.y, ax2.y};
                const f2 any2 = {ay2.x, ay2.x}, afy2 = {ay2.y, ay2.y};
                const f2 anz2 = {az2.x, az2.x}, afz2 = {az2.y, az2.y};
                const float cshift = (delta - mu) * fmaxf(fmaxf(fabsf(inv.x), fabsf(inv.y)), fabsf(inv.z));
#pragma unroll
                for (int k = 0; k < 4; k += 2) {  // slot pairs (k, k+1)
                    auto q2 = [&](unsigned plane) {
                        return (f2){(float)((plane >> (8 * k)) & 255u), (float)((plane >> (8 * k + 8)) & 255u)};
                    };
                    const f2 tnx = __builtin_elementwise_fma(q2(nqx), six2, anx2);
                    const f2 tny = __builtin_elementwise_fma(q2(nqy), siy2, any2);
                    const f2 tnz = __builtin_elementwise_fma(q2(nqz), siz2, anz2);
                    const f2 tfx = __builtin_elementwise_fma(q2(fqx), six2, afx2);
                    const f2 tfy = __builtin_elementwise_fma(q2(fqy), siy2, afy2);
                    const f2 tfz = __builtin_elementwise_fma(q2(fqz), siz2, afz2);
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const float en = fmaxf(fmaxf(tnx[j], tny[j]), tnz[j]);
                        const float tx = fminf(fminf(tfx[j], tfy[j]), tfz[j]);
                        const float e = en - cshift;
                        // (finite here, so a miss is the only +inf key)
                        // (bitwise & / |: no branches per slot)
                        const bool hit = (wd[k + j] != RTG_EXIT) & !((tx < en) | (tx < 0.0f)) & (!io.cull | !(e > tbest));
                        if (COUNT) (anyr ? c_snodes : c_nodes) += wd[k + j] != RTG_EXIT ? 1 : 0;
                        key[k + j] = hit ? e : __builtin_inff();
                    }
                }
            }
            // ascending entry distance (misses sort last); order only affects culling, not results
#define RTG_CSWAP(i, j)                                               \
    if (key[j] < key[i]) {                                           \
        const float tk = key[i]; key[i] = key[j]; key[j] = tk;      \
        const int tw = wd[i]; wd[i] = wd[j]; wd[j] = tw;             \
    }
            RTG_CSWAP(0, 1) RTG_CSWAP(2, 3) RTG_CSWAP(0, 2) RTG_CSWAP(1, 3) RTG_CSWAP(1, 2)
#undef RTG_CSWAP
            // misses carry +inf and sort last
            if (key[0] == __builtin_inff()) {
                cur = RTG_POP;
            } else if (!COUNT && sp + 3 <= STK) {
                // hits are a prefix of the sorted slots: push the h = hits - 1 far ones (far first)
                // with three unconditional LDS writes; entries above sp + h are never read
                const int h = (key[1] != __builtin_inff()) + (key[2] != __builtin_inff()) + (key[3] != __builtin_inff());
                stk[sp][tid] = h == 3 ? wd[3] : (h == 2 ? wd[2] : wd[1]);
                stk[sp + 1][tid] = h == 3 ? wd[2] : wd[1];
                stk[sp + 2][tid] = wd[1];
                sp += h;
                cur = wd[0];
            } else {
#pragma unroll
                for (int k = 3; k >= 1; --k) {
                    if (key[k] != __builtin_inff()) {
                        if (COUNT && sp < STK) kstk[sp][tid] = key[k];
                        if (sp < STK) stk[sp][tid] = wd[k];
                        else io.ovf[(size_t)(sp - STK) * gthreads + gtid] = wd[k];
                        ++sp;
                    }
                }
                cur = wd[0];
            }
        } else if (cur >= 0) {
            if (COUNT) (anyr ? c_snodes : c_nodes) += 2;
            capture(3u, (unsigned)cur);
            const DevNode nd = s.nodes[cur];
            bool hl = slab_exact(nd.a.x, nd.a.y, nd.a.z, nd.a.w, nd.b.x, nd.b.y, o, inv);
            bool hr = slab_exact(nd.b.z, nd.b.w, nd.c.x, nd.c.y, nd.c.z, nd.c.w, o, inv);
            const float el = slab_cull_entry(nd.a.x, nd.a.y, nd.a.z, nd.a.w, nd.b.x, nd.b.y, o, inv, delta);
            const float er = slab_cull_entry(nd.b.z, nd.b.w, nd.c.x, nd.c.y, nd.c.z, nd.c.w, o, inv, delta);
            if (io.cull) {
                hl = hl && !(el > tbest);
                hr = hr && !(er > tbest);
            }
            if (hl && hr) {
                const bool lfirst = !(er < el);
                const int nearw = lfirst ? nd.d.x : nd.d.y;
                const int farw = lfirst ? nd.d.y : nd.d.x;
                if (COUNT && sp < STK) kstk[sp][tid] = -RTG_FLT_MAX;
                if (sp < STK) stk[sp][tid] = farw;
                else io.ovf[(size_t)(sp - STK) * gthreads + gtid] = farw;
                ++sp;
                cur = nearw;
            } else if (hl) {
                cur = nd.d.x;
            } else if (hr) {
                cur = nd.d.y;
            } else {
                cur = RTG_POP;
            }
        }
        // park a reached leaf (one per lane) and keep walking
        if (cur < 0 && cur != RTG_EXIT && cur != RTG_POP && pend == RTG_EXIT) {
            pend = cur;
            cur = RTG_POP;
        } else if (RTG_PEND2 && cur < 0 && cur != RTG_EXIT && cur != RTG_POP && pend2 == RTG_EXIT) {
            pend2 = cur;
            cur = RTG_POP;
        }
        // ---- one pop for every branch: always an LDS read (ds_read, not a flat load through a
        // selected pointer); the global overflow read only for deep entries
        if (cur == RTG_POP) {
            if (COUNT && !anyr && sp > 0) c_pops += 1;
            if (sp == 0) {
                cur = RTG_EXIT;
            } else {
                --sp;
                cur = stk[sp < STK ? sp : 0][tid];
                if (COUNT && !anyr && sp < STK && kstk[sp][tid] > tbest) c_cullpop += 1;
                if (sp >= STK) cur = io.ovf[(size_t)(sp - STK) * gthreads + gtid];
            }
        }
        // leaf phase (wave-uniform): enough parked leaves, or no lane can walk on, or (the queue is
        // dry) any parked leaf: the drain is latency-bound, lanes should not wait for each other
        const unsigned long long pm = __ballot(pend != RTG_EXIT);
        if (__popcll(pm) >= RTG_POSTPONE || __ballot(cur >= 0) == 0 || (drained && pm)) {
            if (COUNT) {
                c_lslots += 64;
                c_lstep += pend != RTG_EXIT ? 1 : 0;
            }
            if (pend != RTG_EXIT) {
                leaf(pend);
                pend = RTG_PEND2 ? pend2 : RTG_EXIT;
                if (RTG_PEND2) pend2 = RTG_EXIT;
                if (anyr && occluded) {
                    cur = RTG_EXIT;
                    sp = 0;
                    if (RTG_PEND2) pend = RTG_EXIT;
                }
            }
        }
    }
    if (RTG_DEBUG && io.wtime && lane == 0) io.wtime[3 * wslot + 2] = __builtin_amdgcn_s_memrealtime();
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            c_nodes += __shfl_down(c_nodes, off);
            c_tris += __shfl_down(c_tris, off);
            c_snodes += __shfl_down(c_snodes, off);
            c_stris += __shfl_down(c_stris, off);
            c_nstep += __shfl_down(c_nstep, off);
            c_lstep += __shfl_down(c_lstep, off);
            c_cullpop += __shfl_down(c_cullpop, off);
            c_pops += __shfl_down(c_pops, off);
            c_lbox += __shfl_down(c_lbox, off);
            c_tails += __shfl_down(c_tails, off);
            c_idle_e += __shfl_down(c_idle_e, off);
            c_idle_ll += __shfl_down(c_idle_ll, off);
            c_idle_lb += __shfl_down(c_idle_lb, off);
            c_idle_r += __shfl_down(c_idle_r, off);
            c_idle_lp += __shfl_down(c_idle_lp, off);
        }
        if (lane == 0) {
            atomicAdd(&io.stats[0], c_nodes);
            atomicAdd(&io.stats[1], c_tris);
            atomicAdd(&io.stats[4], c_snodes);
            atomicAdd(&io.stats[5], c_stris);
            atomicAdd(&io.stats[8], c_slots);
            atomicAdd(&io.stats[9], c_nstep);
            atomicAdd(&io.stats[10], c_lstep);
            atomicAdd(&io.stats[13], c_lslots);
            atomicAdd(&io.stats[11], c_cullpop);
            atomicAdd(&io.stats[12], c_pops);
            atomicAdd(&io.stats[6], (unsigned long long)c_tails);
            atomicAdd(&io.stats[7], c_lbox);
            atomicAdd(&io.stats[15], c_idle_e);
            atomicAdd(&io.stats[16], c_idle_ll);
            atomicAdd(&io.stats[17], c_idle_lb);
            atomicAdd(&io.stats[18], c_idle_r);
            atomicAdd(&io.stats[19], c_idle_lp);
        }
    }
}

// The slice table of the captured launch (trace_slice for k = 0..7: elo, elen, slo, shadow count at
// [k], [8 + k], [16 + k], [24 + k]; [32] the extension index span, [33] / [34] the ray counts).
__global__ void k_cap_slices(TraceIO io, unsigned* tab) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned nc = io.seg_cap ? 8u * io.seg_cap : (io.count ? *io.count : 0u);
    const unsigned n = nc + (io.scount ? *io.scount : 0u);
    unsigned te = 0, ts = 0;
    for (int k = 0; k < 8; ++k) {
        unsigned elo, elen, len;
        trace_slice(io, nc, n, k, elo, elen, len);
        if (!io.fetch8 && k > 0) elo = elen = len = 0;  // one work counter: a single slice (slice 0)
        tab[k] = elo;
        tab[8 + k] = elen;
        tab[16 + k] = elo;
        tab[24 + k] = len - elen;
        te += elen;
        ts += len - elen;
    }
    tab[32] = nc;
    tab[33] = te;
    tab[34] = ts;
}

#if RTG_DEBUG
// ------------------------------------------------------------------ locality-matched ceiling
// Replays the record fetches k_trace made for every ray of one launch (captured in order by
// RTG_OPT_CAPTURE) on the scene's own arrays: the same record types, addresses, per-ray order and
// ray-to-lane grouping, with nothing else in the loop but the fetch of the next chain entry (one
// coalesced uint4 per four steps) and 64 dependent VALU per step, at k_trace's occupancy and with
// its work distribution (8 slice counters by blockIdx % 8, 64-ray pool batches, per-lane refill).
// Each fetch's address depends on the previous record's data (xor with `zero` = 0 at run time), so
// every ray is one dependent chain, as in the walk. Its time is the memory system's time for this
// exact access stream: the ceiling k_trace's time is compared against. Between fetches
// a chain of RTG_REPLAY_VALU dependent FMAs (round 4: 64, which the round-5 walk outran: the ceiling
// must hold less work per fetch than the walk does).
#ifndef RTG_REPLAY_VALU
#define RTG_REPLAY_VALU 8
#endif
__global__ __launch_bounds__(RTG_TB) __attribute__((amdgpu_waves_per_eu(RTG_TRACE_WPE)))
void k_replay(SceneView s, const uint4* cap, const unsigned* cap_len, const unsigned* tab, unsigned cap_n,
              unsigned zero, unsigned* fetch8, unsigned long long* total, float* out) {
    const int lane = lane_id();
    const int slice0 = (int)(blockIdx.x & 7u);
    int slice = slice0, tried = 0;
    const unsigned nc = tab[32];
    unsigned s_elo = tab[slice], s_elen = tab[8 + slice], s_slo = tab[16 + slice], s_len = s_elen + tab[24 + slice];
    unsigned pool_base = 0, pool_left = 0;
    bool drained = false, have = false;
    unsigned ri = 0, k = 0, len = 0, dep = 0;
    uint4 q = make_uint4(0, 0, 0, 0);
    float acc = 0.0f;
    unsigned long long fetches = 0;
    for (;;) {
        const unsigned long long im = __ballot(!have);
        if (im != 0 && !drained) {
            while (pool_left == 0) {
                unsigned b = 0;
                if (lane == 0) b = atomicAdd(fetch8 + 32 * slice, 64u);
                b = __builtin_amdgcn_readfirstlane(b);
                if (b < s_len) {
                    pool_base = b;
                    pool_left = min(64u, s_len - b);
                } else if (++tried == 8) {
                    drained = true;
                    break;
                } else {
                    slice = (slice + 1) & 7;
                    s_elo = tab[slice];
                    s_elen = tab[8 + slice];
                    s_slo = tab[16 + slice];
                    s_len = s_elen + tab[24 + slice];
                }
            }
            if (pool_left > 0) {
                const unsigned pos = prefix_lt(im);
                const unsigned take = min((unsigned)__popcll(im), pool_left);
                if (!have && pos < take) {
                    const unsigned j = pool_base + pos;
                    ri = j < s_elen ? s_elo + j : nc + s_slo + (j - s_elen);
                    len = ri < cap_n ? min(cap_len[ri], (unsigned)RTG_CAP_LEN) : 0u;
                    k = 0;
                    have = len > 0;
                }
                pool_base += take;
                pool_left -= take;
            }
        }
        if (drained && __ballot(have) == 0) break;
        if (!have) continue;
        // the chain entries stream past once: non-temporal, so they do not evict the scene's lines
        // from L2 / MALL (with plain loads the replay's 16 B per 4 fetches made it slower than the
        // round-5 walk on C3 and C4)
        if ((k & 3) == 0) {
            typedef unsigned u4v __attribute__((ext_vector_type(4)));
            const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(cap) + (size_t)(k >> 2) * cap_n + ri);
            q = make_uint4(v.x, v.y, v.z, v.w);
        }
        const unsigned j = k & 3;
        const unsigned e = (j == 0 ? q.x : j == 1 ? q.y : j == 2 ? q.z : q.w) ^ (dep & zero);
        const unsigned type = e >> 30, idx = e & 0x3fffffffu;
        float sum;
        if (type == 0) {
            const float4* r = s.nodesq[idx].q;
            const float4 a = r[0], b = r[1], c = r[2], d = r[3];
            sum = (((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w))) + (((c.x + c.y) + (c.z + c.w)) + ((d.x + d.y) + (d.z + d.w)));
        } else if (type == 1) {
            const float4 a = s.tris48[idx].a, b = s.tris48[idx].b;  // the head: n and v0 decide t
            sum = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
        } else if (type == 2) {
            const float4 a = s.leafbox[2 * idx], b = s.leafbox[2 * idx + 1];
            sum = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
        } else {
            const DevNode nd = s.nodes[idx];
            sum = (((nd.a.x + nd.a.y) + (nd.a.z + nd.a.w)) + ((nd.b.x + nd.b.y) + (nd.b.z + nd.b.w))) +
                  (((nd.c.x + nd.c.y) + (nd.c.z + nd.c.w)) + __int_as_float(nd.d.x ^ nd.d.y));
        }
#pragma unroll
        for (int v = 0; v < RTG_REPLAY_VALU; ++v) sum = __builtin_fmaf(sum, 1.0000001f, (float)v);
        acc += sum;
        dep = __float_as_uint(sum);
        ++fetches;
        if (++k == len) have = false;
    }
    for (int off = 32; off > 0; off >>= 1) fetches += __shfl_down(fetches, off);
    if (lane == 0) atomicAdd(total, fetches);
    if (acc == 1.2345f) out[0] = acc;  // keep the loads
}
#endif

// ------------------------------------------------------------------ generate
// lean (the path tracer): one thread per pixel. renderTile's camera ray goes through the pixel centre
// (Renderer.h:805-808: no jitter, a pinhole camera), so every sample of a pixel casts the same ray
// and finds the same first hit: the bounce-0 traversal traces one ray per pixel (ray_d[lp],
// hits[lp]) and k_shade's bounce 0 reads it for each of the pixel's samples. The rays counted in
// rtg_stats stay the reference's (one per sample); traced_camera_rays counts the traced ones.
// Otherwise (instant radiosity's camera pass, one sample): one thread per path, full path state.
__global__ __launch_bounds__(RTG_TB) void k_generate(ChunkArgs a, PathBufs p) {
    const unsigned pid = blockIdx.x * blockDim.x + threadIdx.x;
    if (a.seg_tiles && pid < 8) {  // path tracer: the paths as queue segments (positions = path ids)
        const unsigned cap = a.seg_tiles * RTG_TB, lo = pid * cap;
        p.ctr[0].ne8[32 * pid] = a.P > lo ? min(cap, a.P - lo) : 0u;
    }
    if (a.seg_tiles && pid == 0) p.ctr[0].n_cam = a.npix;  // the bounce-0 traversal: a ray per pixel
    if (!a.seg_tiles && pid == 0) p.ctr[0].n_ext = a.P;  // instant radiosity's camera pass: one queue
    unsigned lp, sl;  // pixel-major path ids
    if (a.lean) {
        if (pid >= a.npix) return;
        lp = pid;
        sl = 0;
    } else {
        if (pid >= a.P) return;
        split_pid(a, pid, lp, sl);
    }
    const unsigned pixel = a.pixlist[lp];
    const unsigned W = (unsigned)a.cam.width;
    const unsigned x = pixel % W, y = pixel / W;
    const float px = (float)x + 0.5f, py = (float)y + 0.5f;  // renderTile: pixel centre
    // Camera::generateRay
    float xp = px / a.cam.width;
    float yp = 1.0f - (py / a.cam.height);
    xp = (xp * 2.0f) - 1.0f;
    yp = (yp * 2.0f) - 1.0f;
    const float* m = a.cam.ip;
    v3 dir = mk(((xp * m[0] + yp * m[1]) + 1.0f * m[2]) + m[3],
                ((xp * m[4] + yp * m[5]) + 1.0f * m[6]) + m[7],
                ((xp * m[8] + yp * m[9]) + 1.0f * m[10]) + m[11]);
    const float* c = a.cam.cm;
    dir = mk((dir.x * c[0] + dir.y * c[1]) + dir.z * c[2],
             (dir.x * c[4] + dir.y * c[5]) + dir.z * c[6],
             (dir.x * c[8] + dir.y * c[9]) + dir.z * c[10]);
    dir = normalize(dir);
    p.ray_d[pid] = make_float4(dir.x, dir.y, dir.z, 0.0f);  // (lean: pid = lp)
    if (a.lean) return;  // the rest is implied at bounce 0 (k_trace: io.cam_o / identity queue; k_shade)
    p.ray_o[pid] = make_float4(a.cam.ox, a.cam.oy, a.cam.oz, 0.0f);
    p.q[0][pid] = pid;
    p.thr[pid] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    p.rng[pid] = pcg_seed(a.seed, pcg_inc(pixel, a.s0 + sl));
    p.meta[pid] = 1 << 8;  // canHitLight = true
}

// ------------------------------------------------------------------ shade: rtg_shade.hip (k_shade, launch_shade)

// ------------------------------------------------------------------ accumulate
__global__ __launch_bounds__(RTG_TB) void k_accumulate(ChunkArgs a, PathBufs p, float* film) {
    const unsigned lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= a.npix) return;
    const unsigned pixel = a.pixlist[lp];
    float fr = film[(size_t)pixel * 3 + 0], fg = film[(size_t)pixel * 3 + 1], fb = film[(size_t)pixel * 3 + 2];
    for (unsigned sl = 0; sl < a.ns; ++sl) {
        const unsigned pid = lp * a.ns + sl;
        const int nt = p.meta[pid] & 0xff;
        float4 acc = p.contrib[(size_t)(nt - 1) * a.P + pid];
        for (int j = nt - 2; j >= 0; --j) {
            const float4 c = p.contrib[(size_t)j * a.P + pid];
            acc = make_float4(c.x + acc.x, c.y + acc.y, c.z + acc.z, 0.0f);
        }
        fr = fr + acc.x;
        fg = fg + acc.y;
        fb = fb + acc.z;
    }
    film[(size_t)pixel * 3 + 0] = fr;
    film[(size_t)pixel * 3 + 1] = fg;
    film[(size_t)pixel * 3 + 2] = fb;
}

// Several samples per pixel (pid = lp * ns + sl): lane = sample, so the contrib reads are
// contiguous. ns >= 33: one wave per pixel, 64 samples at a time; ns <= 32: one group of
// max(ns, 4) lanes per pixel, as many groups as fit in a wave (C5's 16-sample chunks would otherwise
// leave 3/4 of the lanes idle). Each lane folds its path's right-nested sum; then lanes 0-2 of a pixel's group (R, G, B)
// add its samples to the film in sample order from LDS: the same additions in the same order as
// k_accumulate, so the same bits.
__global__ __launch_bounds__(RTG_TB) void k_accumulate_pm(ChunkArgs a, PathBufs p, float* film) {
    __shared__ float s_acc[RTG_TB / 64][64][4];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const unsigned gw = a.ns < 4 ? 4u : a.ns;          // lanes per pixel group (>= 3: R, G, B folds)
    const unsigned ppw = a.ns <= 32 ? 64u / gw : 1u;   // pixels per wave
    const unsigned grp = ppw > 1 ? (unsigned)lane / gw : 0u;
    const unsigned lp = (blockIdx.x * (RTG_TB / 64) + wave) * ppw + grp;
    const bool active = grp < ppw && lp < a.npix;
    const unsigned pixel = active ? a.pixlist[lp] : 0u;
    const unsigned first = ppw > 1 ? grp * gw : 0u;    // the group's first lane
    const unsigned ch = (unsigned)lane - first;        // the channel this lane folds (0-2)
    float fc = (active && ch < 3) ? film[(size_t)pixel * 3 + ch] : 0.0f;
    const unsigned step = ppw > 1 ? a.ns : 64u;
    for (unsigned s0 = 0; s0 < a.ns; s0 += step) {
        const unsigned sl = s0 + ((unsigned)lane - first);
        float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (active && sl < a.ns) {
            const unsigned pid = lp * a.ns + sl;
            const int nt = p.meta[pid] & 0xff;
            acc = p.contrib[(size_t)(nt - 1) * a.P + pid];
            for (int j = nt - 2; j >= 0; --j) {
                const float4 c = p.contrib[(size_t)j * a.P + pid];
                acc = make_float4(c.x + acc.x, c.y + acc.y, c.z + acc.z, 0.0f);
            }
        }
        s_acc[wave][lane][0] = acc.x;
        s_acc[wave][lane][1] = acc.y;
        s_acc[wave][lane][2] = acc.z;
        __syncthreads();
        const unsigned cnt = min(step, a.ns - s0);
        if (active && ch < 3)
            for (unsigned j = 0; j < cnt; ++j) fc = fc + s_acc[wave][first + j][ch];
        __syncthreads();
    }
    if (active && ch < 3) film[(size_t)pixel * 3 + ch] = fc;
}

// sampleTileWithWeight's splat (Renderer.h:661-670): film += (sum of n samples) / (float)n for the
// listed pixels; tmp holds the per-pixel sums of a scratch render.
__global__ __launch_bounds__(RTG_TB) void k_fold_mean(const unsigned* pixlist, unsigned npix, const float* tmp,
                                                      float count, float* film) {
    const unsigned lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= npix) return;
    const size_t q = (size_t)pixlist[lp] * 3;
    for (int c = 0; c < 3; ++c) film[q + c] = film[q + c] + (tmp[q + c] / count);
}

// BSDF probe: the exact device BSDF code on scripted inputs (unit parity vs RTBase's BSDF classes).
// in: 20 floats per case = kind, int_ior, ext_ior, albedo.rgb (1x1 texture), sN.xyz, wo.xyz, tu, tv,
//     draws[4], pad[2]; out: 11 floats = wi.xyz, refl.rgb, pdf, draws used, evaluate.rgb
__global__ void k_probe_bsdf(const float* in, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* c = in + (size_t)i * 20;
    const int kind = (int)c[0];
    const v3 alb = bilinear(Texels3{c + 3}, 1, 1, c[12], c[13]);  // albedo->sample(tu, tv)
    const frame fr = frame_from(mk(c[6], c[7], c[8]));
    const v3 wo = mk(c[9], c[10], c[11]);
    ScriptSampler smp{c + 14, 4, 0};
    v3 refl;
    float pdf;
    const v3 wi = bsdf_sample(kind, c[1], c[2], alb, fr, wo, smp, refl, pdf);
    const v3 ev = kind <= 1 ? divs_pi(alb) : (kind == 2 ? alb : mk(0.0f, 0.0f, 0.0f));
    float* o = out + (size_t)i * 11;
    o[0] = wi.x; o[1] = wi.y; o[2] = wi.z;
    o[3] = refl.x; o[4] = refl.y; o[5] = refl.z;
    o[6] = pdf;
    o[7] = (float)smp.i;
    o[8] = ev.x; o[9] = ev.y; o[10] = ev.z;
}

// Transcendental probe: the device's include/rtg_math.h on given inputs (parity vs the host glibc).
// fn 0 sinf, 1 cosf, 2 sincosf (out: sin, cos per input), 3 acosf, 4 atan2f (in: y, x per input).
__global__ void k_probe_math(int fn, const float* in, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (fn) {
    case 0: out[i] = rtm_sinf(in[i]); break;
    case 1: out[i] = rtm_cosf(in[i]); break;
    case 2: rtm_sincosf(in[i], &out[2 * (size_t)i], &out[2 * (size_t)i + 1]); break;
    case 3: out[i] = rtm_acosf(in[i]); break;
    default: out[i] = rtm_atan2f(in[2 * (size_t)i], in[2 * (size_t)i + 1]); break;
    }
}

// Per-chunk ray tally: extension + shadow queue lengths of every bounce into stats[2..3]. One wave:
// lane j reads the counters of (bounce, segment) pairs j, j + 64, ... (a lone thread's dependent
// walk over 9 x maxb counters took ~80 us, on the critical path of a 1-spp frame)
__global__ void k_tally(const Counters* ctr, int maxb, unsigned long long* stats) {
    const int lane = threadIdx.x;
    unsigned long long e = 0, sh = 0;
    for (int j = lane; j < maxb * 9; j += 64) {
        const int b = j / 9, k = j % 9;
        if (k == 8) {
            e += ctr[b].n_ext;
            sh += ctr[b].n_shadow;
        } else {  // segmented queues (path tracer)
            e += ctr[b].ne8[32 * k];
            sh += ctr[b].ns8[32 * k];
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        e += __shfl_down(e, off);
        sh += __shfl_down(sh, off);
    }
    if (lane == 0) {
        atomicAdd(&stats[2], e);  // chunks in flight tally concurrently
        atomicAdd(&stats[3], sh);
        atomicAdd(&stats[14], (unsigned long long)ctr[0].n_cam);  // camera rays traced (path tracer)
    }
}

// ================================================================== host side (C-ABI)
thread_local std::string g_err;
static void free_chunk(ChunkSlot& sl) {
    PathBufs& p = sl.pb;
    if (sl.stream) (void)hipStreamSynchronize(sl.stream);  // queued launches may still use the buffers
    (void)hipFree(p.thr); (void)hipFree(p.rng); (void)hipFree(p.meta); (void)hipFree(p.contrib);
    (void)hipFree(p.q[0]); (void)hipFree(p.q[1]); (void)hipFree(p.hits); (void)hipFree(p.shq); (void)hipFree(p.ctr);
    (void)hipFree(p.ray_o); (void)hipFree(p.ray_d);
    (void)hipFree(p.thr2); (void)hipFree(p.rng2); (void)hipFree(p.ray_o2); (void)hipFree(p.ray_d2);
    (void)hipFree(p.sh_o); (void)hipFree(p.sh_d); (void)hipFree(p.sh_c);
    p = PathBufs{};
    sl.cap_P = 0;
    sl.cap_maxb = 0;
}

// bytes of path state per path: 200 B of payload and queue arrays, 16 B per contribution plane, and
// 8 B for the id queues (light tracer / instant radiosity only)
static size_t path_bytes(int planes, bool queues) { return (size_t)200 + (size_t)16 * (size_t)planes + (queues ? 8u : 0u); }
static size_t slot_bytes(const ChunkSlot& sl) { return sl.cap_P * path_bytes(sl.cap_maxb, sl.pb.q[0] != nullptr); }

#ifndef RTG_SLOT_STREAMS
#define RTG_SLOT_STREAMS 1  // 0: plain streams, 1: one priority per slot
#endif
// Plain streams beyond GPU_MAX_HW_QUEUES share HSA queues, and two slots on one queue run in turn
// (queued 1-spp frames 2.93 ms each). Streams of different priorities (1) get queues of their own:
// 2.28 ms. (Full-CU-mask streams also do, 2.21 ms, but destroying them deadlocked the runtime after a
// few handles (ROCm 7.2, tools/r04_churn.py) and kept alive in a per-device pool they crashed the
// process at exit under rocprofv3: removed)
static int ensure_stream(rtg_handle* h, ChunkSlot& sl) {
    if (!sl.stream) {
        const int k = (int)(&sl - h->slot);
        if (RTG_SLOT_STREAMS == 1) {
            int lo = 0, hi = 0;
            HIPOK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPOK(hipStreamCreateWithPriority(&sl.stream, hipStreamNonBlocking, k == 0 ? lo : k == 1 ? hi : (lo + hi) / 2));
        } else {
            HIPOK(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
        }
    }
    if (!sl.fold) HIPOK(hipEventCreateWithFlags(&sl.fold, hipEventDisableTiming));
    return RTG_OK;
}

int ensure_chunk(rtg_handle* h, ChunkSlot& sl, size_t P, int maxb, bool queues) {
    int rc;
    if ((rc = ensure_stream(h, sl))) return rc;
    PathBufs& p = sl.pb;
    if (P <= sl.cap_P && maxb <= sl.cap_maxb) {
        if (queues && !p.q[0]) {
            if (sl.stream) HIPOK(hipStreamSynchronize(sl.stream));
            HIPOK(hipMalloc((void**)&p.q[0], sl.cap_P * sizeof(unsigned)));
            HIPOK(hipMalloc((void**)&p.q[1], sl.cap_P * sizeof(unsigned)));
        }
        return RTG_OK;
    }
    free_chunk(sl);
    const size_t Q = queue_slots(P);  // arrays indexed by queue position (segmented queues)
    HIPOK(hipMalloc((void**)&p.thr, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.rng, Q * sizeof(unsigned long long)));
    HIPOK(hipMalloc((void**)&p.meta, P * sizeof(int)));
    HIPOK(hipMalloc((void**)&p.contrib, P * (size_t)maxb * sizeof(float4)));
    if (queues) {
        HIPOK(hipMalloc((void**)&p.q[0], P * sizeof(unsigned)));
        HIPOK(hipMalloc((void**)&p.q[1], P * sizeof(unsigned)));
    }
    HIPOK(hipMalloc((void**)&p.shq, Q * sizeof(unsigned)));
    HIPOK(hipMalloc((void**)&p.hits, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.ray_o, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.ray_d, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.thr2, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.rng2, Q * sizeof(unsigned long long)));
    HIPOK(hipMalloc((void**)&p.ray_o2, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.ray_d2, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.sh_o, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.sh_d, Q * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.sh_c, P * sizeof(float4)));
    HIPOK(hipMalloc((void**)&p.ctr, (size_t)(maxb + 1) * sizeof(Counters)));
    sl.cap_P = P;
    sl.cap_maxb = maxb;
    return RTG_OK;
}

int ensure_ovf(rtg_handle* h, ChunkSlot& sl) {
    int grid = std::max(std::max(h->trace_blocks, h->trace_blocks_count),
                        std::max(h->trace_blocks_small, h->trace_blocks_small_count));
    // deepest stack: one entry per BVH2 level, or up to 3 per wide level (each wide level descends
    // at least one BVH2 level); the small-scene variant keeps fewer entries in LDS
    size_t deep = std::max<size_t>(h->bvh_depth, (size_t)h->wide_depth * 3) + 2;
    const size_t lds = std::min(RTG_STACK, RTG_STACK_SMALL);
    size_t levels = deep > lds ? deep - lds : 1;
    size_t need = levels * (size_t)grid * RTG_TTB;
    if (need <= sl.cap_ovf) return RTG_OK;
    if (sl.stream) HIPOK(hipStreamSynchronize(sl.stream));
    (void)hipFree(sl.d_ovf);
    sl.d_ovf = nullptr;
    HIPOK(hipMalloc((void**)&sl.d_ovf, need * sizeof(int)));
    sl.cap_ovf = need;
    return RTG_OK;
}

int flush_pending(rtg_handle* h) {
    if (!h->pend_n) return RTG_OK;
    const uint32_t first = h->pend_first, n = h->pend_n;
    h->pend_n = 0;
    const bool all = h->pend_key.size() == 1 && h->pend_key[0] == 0xffffffffu;
    const std::vector<uint32_t> key = h->pend_key;
    const int rc = render_impl(h, first, n, h->pend_seed, all ? nullptr : key.data(), all ? 0u : (uint32_t)key.size(),
                               h->stream, true, false);
    // rtg_render_async counted the frames in Film::SPP when they were queued; frames whose issue
    // failed never reach the film (chunks issued before the failure may have: the film is then
    // partial, and the error says so)
    if (rc) h->spp -= std::min(h->spp, n);
    return rc;
}

int join_frames(rtg_handle* h) {
    if (int rc = flush_pending(h)) return rc;
    if (!h->inflight) return RTG_OK;
    h->inflight = false;
    HIPOK(hipStreamWaitEvent(h->stream, h->last_fold, 0));
    HIPOK(hipEventRecord(h->ev[1], h->stream));  // the end of the queued run (rtg_stats::render_ms)
    return RTG_OK;
}

static float host_bits_f(int v) { float f; std::memcpy(&f, &v, 4); return f; }

// Compressed 4-wide node: per axis the smallest power-of-two step with origin + 255*step >= max,
// then each slot bound rounded outward and verified with the device's decode (qdecode), so the
// decoded box contains the exact one. Returns false if a step would leave the exponent range.
static bool encode_qnode(const float* bounds, const std::vector<int>& slots, const int32_t* words, DevNodeQ& out) {
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = bounds[(size_t)slots[0] * 6 + a];
        hi[a] = bounds[(size_t)slots[0] * 6 + 3 + a];
        for (int k = 1; k < (int)slots.size(); ++k) {
            lo[a] = std::min(lo[a], bounds[(size_t)slots[k] * 6 + a]);
            hi[a] = std::max(hi[a], bounds[(size_t)slots[k] * 6 + 3 + a]);
        }
    }
    unsigned planes[6] = {0, 0, 0, 0, 0, 0};
    unsigned bexp[3];
    for (int a = 0; a < 3; ++a) {
        const double ext = (double)hi[a] - (double)lo[a];
        int e = ext > 0 ? (int)std::ceil(std::log2(ext / 255.0)) : -126;
        e = std::max(e, -126);
        for (;; ++e) {
            if (e > 119) return false;
            if (rtgd::qdecode(lo[a], 255u, 0, host_bits_f((e + 127) << 23)) >= hi[a]) break;
        }
        bexp[a] = (unsigned)(e + 127);
        const float sc = host_bits_f((e + 127) << 23);
        for (int k = 0; k < (int)slots.size(); ++k) {
            const float mn = bounds[(size_t)slots[k] * 6 + a], mx = bounds[(size_t)slots[k] * 6 + 3 + a];
            int ql = (int)std::floor(((double)mn - (double)lo[a]) / std::ldexp(1.0, e));
            int qh = (int)std::ceil(((double)mx - (double)lo[a]) / std::ldexp(1.0, e));
            ql = std::min(std::max(ql, 0), 255);
            qh = std::min(std::max(qh, 0), 255);
            while (ql > 0 && rtgd::qdecode(lo[a], (unsigned)ql, 0, sc) > mn) --ql;
            while (qh < 255 && rtgd::qdecode(lo[a], (unsigned)qh, 0, sc) < mx) ++qh;
            if (rtgd::qdecode(lo[a], (unsigned)ql, 0, sc) > mn || rtgd::qdecode(lo[a], (unsigned)qh, 0, sc) < mx)
                return false;
            planes[a] |= (unsigned)ql << (8 * k);
            planes[3 + a] |= (unsigned)qh << (8 * k);
        }
    }
    auto uf = [](unsigned v) { float f; std::memcpy(&f, &v, 4); return f; };
    out.q[0] = make_float4(lo[0], lo[1], lo[2], uf(bexp[0] | (bexp[1] << 8) | (bexp[2] << 16)));
    out.q[1] = make_float4(uf(planes[0]), uf(planes[1]), uf(planes[2]), uf(planes[3]));
    out.q[2] = make_float4(uf(planes[4]), uf(planes[5]), host_bits_f(words[0]), host_bits_f(words[1]));
    out.q[3] = make_float4(host_bits_f(words[2]), host_bits_f(words[3]), 0.0f, 0.0f);
    return true;
}
static float host_dot(const float* a, const float* b) { return ((a[0] * b[0]) + (a[1] * b[1])) + (a[2] * b[2]); }
static void host_cross(const float* a, const float* b, float* o) {
    o[0] = (a[1] * b[2]) - (a[2] * b[1]);
    o[1] = (a[2] * b[0]) - (a[0] * b[2]);
    o[2] = (a[0] * b[1]) - (a[1] * b[0]);
}

// Own binary SAH tree over the scene's triangles (or the reference's leaves), in the descriptor's node
// format (links {left, right, start, end}, bounds {min xyz, max xyz}; node 0 is the root). Internal
// boxes are float min/max unions, so containment is exact and the wide walk built from this tree
// reaches every primitive whose box the ray passes; k_trace's leaf-box test keeps reachability the
// reference's. The reference splits along the longest axis only (Geometry.h:343-386); this build
// tries all three: full SAH sweep below 2048 primitives, 64 centroid bins per axis above.
#ifndef RTG_TRI_LEAVES
#define RTG_TRI_LEAVES 1    // 0: the primitives are the reference leaves (rounds 2-4)
#endif
static bool rebuild_over_leaves(const rtg_scene_desc* d, std::vector<int32_t>& lk, std::vector<float>& bd) {
    // Primitives (round 5): every triangle alone, its box inflated by 2^-17 of the scene scale and
    // rounded outward (a hit that rayIntersect reports lies within rounding of its triangle, far inside
    // that margin plus the slot test's), so a wide leaf slot holds one triangle
    // and its box is the triangle's, not its reference leaf's. C3: triangle tests per ray 11.7 -> 6.4,
    // node steps 25.3 -> 27.0, traversal -12.5 %; C4 -40 %. (Keeping two consecutive triangles in one
    // slot when their union box is no larger than their two boxes measured slower everywhere, even on
    // quads: the leaf's two tests are one dependent chain.) Acceptance is unchanged: a candidate hit
    // counts only if its reference leaf box passes the exact test (leafbox). Non-finite positions, or
    // RTG_TRI_LEAVES=0: the reference leaves, kept whole.
    std::vector<float> pbox;
    std::vector<std::array<int32_t, 4>> plink;
    bool tri_ok = RTG_TRI_LEAVES != 0;
    for (size_t k = 0; tri_ok && k < (size_t)d->n_tris * 9; ++k) tri_ok = std::isfinite(d->positions[k]);
    if (tri_ok) {
        float scale = 0.0f;
        for (int k = 0; k < 6; ++k)
            if (std::isfinite(d->node_bounds[k])) scale = std::max(scale, std::fabs(d->node_bounds[k]));
        const double eps = std::ldexp((double)scale, -17);
        for (uint32_t t = 0; t < d->n_tris; ++t) {
            const float* P = d->positions + (size_t)t * 9;
            for (int a = 0; a < 3; ++a) {
                const double lo = std::min(std::min(P[a], P[3 + a]), P[6 + a]) - eps;
                pbox.push_back(std::nextafter((float)lo, -INFINITY));
            }
            for (int a = 0; a < 3; ++a) {
                const double hi = std::max(std::max(P[a], P[3 + a]), P[6 + a]) + eps;
                pbox.push_back(std::nextafter((float)hi, INFINITY));
            }
            plink.push_back({-1, -1, (int32_t)t, (int32_t)t + 1});
        }
    } else {
        for (uint32_t i = 0; i < d->n_nodes; ++i) {
            const int32_t* L = d->node_links + (size_t)i * 4;
            if (L[0] >= 0) continue;
            pbox.insert(pbox.end(), d->node_bounds + (size_t)i * 6, d->node_bounds + (size_t)i * 6 + 6);
            plink.push_back({L[0], L[1], L[2], L[3]});
        }
    }
    const size_t n = plink.size();
    if (n < 2) return false;
    auto box = [&](int p) { return pbox.data() + (size_t)p * 6; };
    std::vector<float> cen(n * 3);
    for (size_t p = 0; p < n; ++p)
        for (int a = 0; a < 3; ++a) cen[p * 3 + a] = 0.5f * (box((int)p)[a] + box((int)p)[a + 3]);
    struct Bx {
        float b[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
        void add(const float* o) {
            for (int a = 0; a < 3; ++a) { b[a] = std::min(b[a], o[a]); b[a + 3] = std::max(b[a + 3], o[a + 3]); }
        }
        double area() const {
            if (b[0] > b[3]) return 0.0;
            const double x = (double)b[3] - b[0], y = (double)b[4] - b[1], z = (double)b[5] - b[2];
            return x * y + y * z + z * x;
        }
    };
    // SAH weight of a leaf: its triangle count (1-2); full sweep below 2048 leaves, 64 centroid
    // bins per axis above (a full sweep to 16384 leaves or 256 bins measured no better)
    const int sweep_max = RTG_SAH_SWEEP, nbins = RTG_SAH_BINS;
    std::vector<double> wt(n), pre;
    for (size_t p = 0; p < n; ++p) wt[p] = (double)(plink[p][3] - plink[p][2]);
    std::vector<int> idx(n);
    for (size_t p = 0; p < n; ++p) idx[p] = (int)p;
    lk.assign((2 * n - 1) * 4, -1);
    bd.assign((2 * n - 1) * 6, 0.0f);
    int next = 1;
    std::vector<std::array<int, 4>> st{{0, 0, (int)n, 0}};  // node id, range [lo, hi) of idx, depth
    std::vector<Bx> suf;
    while (!st.empty()) {
        auto [node, lo, hi, dep] = st.back();
        st.pop_back();
        if (dep > 96) return false;  // degenerate SAH chain: keep the reference tree (bounded stacks)
        const int m = hi - lo;
        Bx all;
        for (int p = lo; p < hi; ++p) all.add(box(idx[p]));
        std::memcpy(&bd[(size_t)node * 6], all.b, sizeof(all.b));
        if (m == 1) {
            std::memcpy(&lk[(size_t)node * 4], plink[idx[lo]].data(), 4 * sizeof(int32_t));
            continue;
        }
        double best = INFINITY;
        int bax = -1, bsplit = lo + m / 2;  // fallback: median of the current order
        int bbin = 0;
        if (m <= sweep_max) {
            for (int a = 0; a < 3; ++a) {
                std::sort(idx.begin() + lo, idx.begin() + hi, [&](int x, int y) {
                    return cen[x * 3 + a] < cen[y * 3 + a] || (cen[x * 3 + a] == cen[y * 3 + a] && x < y);
                });
                suf.assign(m + 1, Bx());
                for (int p = m - 1; p >= 0; --p) { suf[p] = suf[p + 1]; suf[p].add(box(idx[lo + p])); }
                pre.assign(m + 1, 0.0);
                for (int p = 0; p < m; ++p) pre[p + 1] = pre[p] + wt[idx[lo + p]];
                Bx left;
                for (int p = 1; p < m; ++p) {
                    left.add(box(idx[lo + p - 1]));
                    const double c = left.area() * pre[p] + suf[p].area() * (pre[m] - pre[p]);
                    if (c < best) { best = c; bax = a; bsplit = lo + p; }
                }
            }
            if (bax >= 0) {
                std::sort(idx.begin() + lo, idx.begin() + hi, [&](int x, int y) {
                    return cen[x * 3 + bax] < cen[y * 3 + bax] || (cen[x * 3 + bax] == cen[y * 3 + bax] && x < y);
                });
            }
        } else {
            const int NB = nbins;
            Bx cb;
            for (int p = lo; p < hi; ++p) {
                const float* c = &cen[(size_t)idx[p] * 3];
                const float cc[6] = {c[0], c[1], c[2], c[0], c[1], c[2]};
                cb.add(cc);
            }
            for (int a = 0; a < 3; ++a) {
                const float ext = cb.b[a + 3] - cb.b[a];
                if (!(ext > 0.0f)) continue;
                std::vector<Bx> bins(NB), right(NB + 1);
                std::vector<double> cnt(NB, 0.0), rc(NB + 1, 0.0);
                for (int p = lo; p < hi; ++p) {
                    const int b = std::min(NB - 1, (int)((cen[(size_t)idx[p] * 3 + a] - cb.b[a]) / ext * NB));
                    bins[b].add(box(idx[p]));
                    cnt[b] += wt[idx[p]];
                }
                for (int b = NB - 1; b >= 0; --b) { right[b] = right[b + 1]; right[b].add(bins[b].b); rc[b] = rc[b + 1] + cnt[b]; }
                Bx left;
                double lc = 0;
                for (int b = 1; b < NB; ++b) {
                    left.add(bins[b - 1].b);
                    lc += cnt[b - 1];
                    if (lc == 0 || rc[b] == 0) continue;
                    const double c = left.area() * lc + right[b].area() * rc[b];
                    if (c < best) { best = c; bax = a; bbin = b; }
                }
            }
            if (bax >= 0) {
                const float ext = cb.b[bax + 3] - cb.b[bax];
                auto mid = std::partition(idx.begin() + lo, idx.begin() + hi, [&](int x) {
                    return std::min(NB - 1, (int)((cen[(size_t)x * 3 + bax] - cb.b[bax]) / ext * NB)) < bbin;
                });
                bsplit = (int)(mid - idx.begin());
                if (bsplit == lo || bsplit == hi) bsplit = lo + m / 2;
            }
        }
        const int l = next++, r = next++;
        lk[(size_t)node * 4] = l;
        lk[(size_t)node * 4 + 1] = r;
        lk[(size_t)node * 4 + 2] = lk[(size_t)node * 4 + 3] = 0;
        st.push_back({r, bsplit, hi, dep + 1});
        st.push_back({l, lo, bsplit, dep + 1});
    }
    return next == (int)(2 * n - 1);
}

extern "C" {

int32_t rtg_abi_version(void) { return RTG_ABI_VERSION; }
#ifndef RTG_BUILD_ID
#define RTG_BUILD_ID "unknown"
#endif
// build.py passes the hash of the sources, headers and flags (source_hash("device")); the tagged
// copy lets the build find the id in the file without loading it
static const char k_build_tag[] __attribute__((used)) = "rtg-build-id:" RTG_BUILD_ID;
const char* rtg_build_id(void) { return k_build_tag + 13; }
const char* rtg_last_error(void) { return g_err.c_str(); }

int rtg_device_count(int* count) {
    if (!count) return RTG_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RTG_OK;
}

}  // extern "C"

// The host half of rtg_create: the descriptor (the flattened reference Scene) turned into the device
// records. No HIP calls: a group builds this once and uploads it to every device in parallel.
int prepare_scene(const rtg_scene_desc* d, HostScene& hs) {
    if (d->n_lights == 0) {
        g_err = "scene has no lights (RTBase's Scene::sampleLight indexes an empty list: Scene.h:137-138)";
        return RTG_ERR_NO_LIGHTS;
    }
    const uint32_t nt = d->n_tris;

    // ---- triangles: Triangle::init (Geometry.h:72-83) + gNormal (:127-130)
    std::vector<DevTri48> tris48(nt);
    std::vector<DevShade> shade(nt);
    std::vector<float> tri_area(nt), tri_gn(nt * 3);
    for (uint32_t i = 0; i < nt; ++i) {
        const float* P = d->positions + (size_t)i * 9;
        const float *v0 = P, *v1 = P + 3, *v2 = P + 6;
        float e1[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
        float e2[3] = {v0[0] - v2[0], v0[1] - v2[1], v0[2] - v2[2]};
        float c[3];
        host_cross(e1, e2, c);
        float l = 1.0f / std::sqrt(((c[0] * c[0]) + (c[1] * c[1])) + (c[2] * c[2]));
        float n[3] = {c[0] * l, c[1] * l, c[2] * l};
        tri_area[i] = std::sqrt(((c[0] * c[0]) + (c[1] * c[1])) + (c[2] * c[2])) * 0.5f;
        const float* N = d->normals + (size_t)i * 9;
        float s = host_dot(N, n) > 0 ? 1.0f : -1.0f;
        for (int k = 0; k < 3; ++k) tri_gn[i * 3 + k] = n[k] * s;
        tris48[i].a = make_float4(n[0], n[1], n[2], v0[0]);
        tris48[i].b = make_float4(v0[1], v0[2], v1[0], v1[1]);
        tris48[i].c = make_float4(v1[2], v2[0], v2[1], v2[2]);
        const float* U = d->uvs + (size_t)i * 6;
        if (d->material[i] >= d->n_materials) { g_err = "triangle material index out of range"; return RTG_ERR_ARG; }
        shade[i].a = make_float4(N[0], N[1], N[2], N[3]);
        shade[i].b = make_float4(N[4], N[5], N[6], N[7]);
        shade[i].c = make_float4(N[8], U[0], U[1], U[2]);
        shade[i].d = make_float4(U[3], U[4], U[5], host_bits_f((int)d->material[i]));
    }
    // ---- BVH: reference DFS nodes -> child-pair internal nodes
    const uint32_t nn = d->n_nodes;
    if (nn == 0) { g_err = "BVH has no nodes"; return RTG_ERR_ARG; }
    std::vector<int> internal_id(nn, -1);
    int n_internal = 0;
    for (uint32_t i = 0; i < nn; ++i)
        if (d->node_links[i * 4 + 0] >= 0) internal_id[i] = n_internal++;
    auto word = [&](int node, int& out) -> bool {
        const int32_t* L = d->node_links + (size_t)node * 4;
        if (L[0] >= 0) { out = internal_id[node]; return true; }
        int cnt = L[3] - L[2];
        if (cnt < 1 || cnt > 2 || L[2] < 0 || (uint32_t)L[3] > nt) return false;
        out = ~(L[2] * RTG_LEAF_SPAN + (cnt - 1));
        return true;
    };
    std::vector<DevNode> nodes(std::max(n_internal, 1));
    uint32_t depth = 0;
    {
        std::vector<std::pair<int, uint32_t>> st{{0, 0}};
        while (!st.empty()) {
            auto [i, dep] = st.back();
            st.pop_back();
            depth = std::max(depth, dep);
            const int32_t* L = d->node_links + (size_t)i * 4;
            if (L[0] < 0) continue;
            if (L[0] >= (int)nn || L[1] < 0 || L[1] >= (int)nn) { g_err = "bad BVH link"; return RTG_ERR_ARG; }
            const float* bl = d->node_bounds + (size_t)L[0] * 6;
            const float* br = d->node_bounds + (size_t)L[1] * 6;
            DevNode& dn = nodes[internal_id[i]];
            dn.a = make_float4(bl[0], bl[1], bl[2], bl[3]);
            dn.b = make_float4(bl[4], bl[5], br[0], br[1]);
            dn.c = make_float4(br[2], br[3], br[4], br[5]);
            int wl, wr;
            if (!word(L[0], wl) || !word(L[1], wr)) {
                g_err = "BVH leaf with other than 1-2 triangles (MAXNODE_TRIANGLES = 2)";
                return RTG_ERR_ARG;
            }
            dn.d = make_int4(wl, wr, 0, 0);
            st.push_back({L[1], dep + 1});
            st.push_back({L[0], dep + 1});
        }
    }
    hs.bvh_depth = depth;
    int root_word = RTG_EXIT;
    if (nt > 0) {
        if (!word(0, root_word)) { g_err = "bad BVH root"; return RTG_ERR_ARG; }
    }
    // ---- wide collapse: each node's slots are a cut of the BVH2 subtree below it, grown by
    // repeatedly opening the internal slot of largest surface area (leaves stay slots). Exact
    // boxes are kept, so reachability is the reference's (see k_trace).
    std::vector<DevNodeQ> nodesq;
    bool qok = true;
    int root_wordw = root_word;
    bool finite = true;
    for (size_t k = 0; k < (size_t)nn * 6; ++k) finite = finite && std::isfinite(d->node_bounds[k]);
    // Skipping levels is exact only if every child box lies inside its parent's (true for
    // Scene::build's bounds; checked so that a foreign descriptor degrades to the BVH2 walk).
    for (uint32_t i = 0; finite && i < nn; ++i) {
        const int32_t* L = d->node_links + (size_t)i * 4;
        if (L[0] < 0) continue;
        const float* P = d->node_bounds + (size_t)i * 6;
        for (int c : {L[0], L[1]}) {
            const float* Cb = d->node_bounds + (size_t)c * 6;
            for (int q = 0; q < 3; ++q) finite = finite && Cb[q] >= P[q] && Cb[q + 3] <= P[q + 3];
        }
    }
    if (nt > 0 && finite && d->node_links[0] >= 0) {
        // the tree the wide nodes are cut from: an own SAH tree over the reference's leaves
        // (rebuild_over_leaves), or the reference BVH2 when that tree cannot be built
        std::vector<int32_t> rlk;
        std::vector<float> rbd;
        const bool rebuilt = (RTG_SBVH && build_sbvh(d, rlk, rbd)) || rebuild_over_leaves(d, rlk, rbd);
        const int32_t* LK = rebuilt ? rlk.data() : d->node_links;
        const float* BD = rebuilt ? rbd.data() : d->node_bounds;
        const uint32_t nn = rebuilt ? (uint32_t)(rlk.size() / 4) : d->n_nodes;
        auto wordw = [&](int node, int& out) -> bool {  // leaf word (leaves are the reference's)
            const int32_t* L = LK + (size_t)node * 4;
            const int cnt = L[3] - L[2];
            if (L[0] >= 0 || cnt < 1 || cnt > 2 || L[2] < 0 || (uint32_t)L[3] > nt) return false;
            out = ~(L[2] * RTG_LEAF_SPAN + (cnt - 1));
            return true;
        };
        hs.rebuilt = rebuilt;
        auto internal = [&](int i) { return LK[(size_t)i * 4] >= 0; };
        auto area = [&](int i) {
            const float* b = BD + (size_t)i * 6;
            const double x = b[3] - b[0], y = b[4] - b[1], z = b[5] - b[2];
            return x * y + y * z + z * x;
        };
        // the slots of the wide node made from BVH2 node n2: a cut of its subtree below it
        auto cut = [&](int n2) {
            std::vector<int> slots;
            slots = {LK[(size_t)n2 * 4], LK[(size_t)n2 * 4 + 1]};
            while ((int)slots.size() < 4) {
                int best_k = -1;
                for (int k = 0; k < (int)slots.size(); ++k)
                    if (internal(slots[k]) && (best_k < 0 || area(slots[k]) > area(slots[best_k]))) best_k = k;
                if (best_k < 0) break;
                const int c = slots[best_k];
                slots[best_k] = LK[(size_t)c * 4];
                slots.push_back(LK[(size_t)c * 4 + 1]);
            }
            return slots;
        };
        nodesq.emplace_back();
        root_wordw = 0;
        std::vector<std::array<int, 3>> work{{0, 0, 1}};  // BVH2 node, wide node, wide level
        while (!work.empty()) {
            auto [n2, nw, lvl] = work.back();
            work.pop_back();
            hs.wide_depth = std::max(hs.wide_depth, (uint32_t)lvl);
            const std::vector<int> slots = cut(n2);
            int32_t wq[4] = {RTG_EXIT, RTG_EXIT, RTG_EXIT, RTG_EXIT};
            for (int k = 0; k < (int)slots.size(); ++k) {
                if (internal(slots[k])) {
                    wq[k] = (int)nodesq.size();
                    nodesq.emplace_back();
                    work.push_back({slots[k], wq[k], lvl + 1});
                } else if (!wordw(slots[k], wq[k])) {
                    g_err = "bad BVH leaf";
                    return RTG_ERR_ARG;
                }
            }
            if (!encode_qnode(BD, slots, wq, nodesq[nw])) { qok = false; break; }
        }
    }
    float cull_scale = 0.0f;
    for (int k = 0; k < 6; ++k)
        if (std::isfinite(d->node_bounds[k])) cull_scale = std::max(cull_scale, std::fabs(d->node_bounds[k]));
    // the compressed walk's rounding margin is stated relative to the scene scale (k_trace)
    hs.usew = finite && qok && nt > 0 && cull_scale >= 0x1p-60f && cull_scale <= 0x1p60f;
    // exact leaf boxes per triangle (compressed walk: candidate hits re-test their leaf)
    std::vector<float4> leafbox(std::max<size_t>((size_t)nt * 2, 2));
    for (uint32_t i = 0; i < nn; ++i) {
        const int32_t* L = d->node_links + (size_t)i * 4;
        if (L[0] >= 0) continue;
        const float* b = d->node_bounds + (size_t)i * 6;
        for (int t = L[2]; t < L[3]; ++t) {
            leafbox[2 * (size_t)t] = make_float4(b[0], b[1], b[2], b[3]);
            leafbox[2 * (size_t)t + 1] = make_float4(b[4], b[5], 0.0f, 0.0f);
        }
    }
    // (RTG_SMALL_LB 0: the leaf boxes stay in global memory, read once per candidate hit)
    const bool small = hs.usew && nodesq.size() * 4 + (size_t)nt * (RTG_SMALL_LB ? 5 : 3) <= RTG_SMALL_F4;
    float scale = 0.0f;
    for (int k = 0; k < 6; ++k) {
        float v = std::fabs(d->node_bounds[k]);
        if (std::isfinite(v)) scale = std::max(scale, v);
    }
    // small scenes: the image k_trace<.., SMALL> copies into LDS (wide nodes | triangles | leaf boxes)
    if (small) {
        hs.img.clear();
        for (const DevNodeQ& q : nodesq) hs.img.insert(hs.img.end(), q.q, q.q + 4);
        hs.img_tri = (int)hs.img.size();
        for (const DevTri48& t : tris48) hs.img.insert(hs.img.end(), {t.a, t.b, t.c});
        hs.img_lb = (int)hs.img.size();
        if (RTG_SMALL_LB) hs.img.insert(hs.img.end(), leafbox.begin(), leafbox.begin() + (size_t)nt * 2);
    }
    // ---- materials, textures, lights
    std::vector<DevMat> mats(d->n_materials);
    for (uint32_t i = 0; i < d->n_materials; ++i) {
        const rtg_material& m = d->materials[i];
        if (m.texture < 0 || (uint32_t)m.texture >= d->n_textures) { g_err = "material texture out of range"; return RTG_ERR_ARG; }
        mats[i].kind = m.kind;
        mats[i].two_sided = m.two_sided;
        mats[i].tex = m.texture;
        const float lm = ((0.2126f * m.emission[0]) + (0.7152f * m.emission[1])) + (0.0722f * m.emission[2]);
        mats[i].is_light = lm > 0 ? 1 : 0;
        mats[i].int_ior = m.int_ior;
        mats[i].ext_ior = m.ext_ior;
        mats[i].emission = make_float4(m.emission[0], m.emission[1], m.emission[2], 0.0f);
    }
    std::vector<DevTex> texinfo(d->n_textures);
    std::vector<float> texels;
    for (uint32_t i = 0; i < d->n_textures; ++i) {
        const rtg_texture& t = d->textures[i];
        if (t.width <= 0 || t.height <= 0 || !t.texels) { g_err = "empty texture"; return RTG_ERR_ARG; }
        texinfo[i] = DevTex{(int)(texels.size() / 4), t.width, t.height, 0};
        for (size_t j = 0; j < (size_t)t.width * t.height; ++j)  // RGB + pad: one 16-B load per texel
            texels.insert(texels.end(), {t.texels[3 * j], t.texels[3 * j + 1], t.texels[3 * j + 2], 0.0f});
    }
    if (d->env_texture >= (int)d->n_textures) { g_err = "env texture out of range"; return RTG_ERR_ARG; }
    // textures whose texels all have the same bits (1x1, or constant like C3's environment): the
    // kernels' bilinear taps use the first texel instead of four dependent fetches (the same operands)
    std::vector<char> uniform_tex(d->n_textures, 1);
    for (uint32_t i = 0; i < d->n_textures; ++i) {
        const rtg_texture& t = d->textures[i];
        const size_t n = (size_t)t.width * t.height;
        for (size_t j = 1; j < n && uniform_tex[i]; ++j) {
            if (!RTG_UNIFORM_TEX) { uniform_tex[i] = 0; break; }  // (A/B: only 1x1 textures)
            uniform_tex[i] = std::memcmp(t.texels + 3 * j, t.texels, 3 * sizeof(float)) == 0;
        }
    }
    for (uint32_t i = 0; i < d->n_materials; ++i) {  // texture offset and size into the material record
        const DevTex& t = texinfo[mats[i].tex];
        if (t.w > 0xffff || t.h > 0xffff) { g_err = "texture larger than 65535 texels per side"; return RTG_ERR_ARG; }
        mats[i].tex = t.off;
        mats[i].tex_wh = (int)((unsigned)t.w | ((unsigned)t.h << 16));
        mats[i].uniform = uniform_tex[(size_t)(&t - texinfo.data())] ? 1 : 0;
        mats[i].texel0 = make_float4(texels[(size_t)t.off * 4], texels[(size_t)t.off * 4 + 1], texels[(size_t)t.off * 4 + 2], 0.0f);
    }
    // Identical material records merged (a scene file gives every instance its own BSDF: bathroom_f
    // has 852 for 24 distinct ones), so k_shade can hold the table in LDS; the triangles' shading
    // records are remapped. Same record, same arithmetic: the output does not change.
    {
        std::vector<DevMat> uniq;
        std::vector<int> remap(mats.size());
        for (size_t i = 0; i < mats.size(); ++i) {
            size_t j = 0;
            while (j < uniq.size() && std::memcmp(&uniq[j], &mats[i], sizeof(DevMat)) != 0) ++j;
            if (j == uniq.size()) uniq.push_back(mats[i]);
            remap[i] = (int)j;
        }
        for (uint32_t i = 0; i < nt; ++i) shade[i].d.w = host_bits_f(remap[d->material[i]]);
        mats.swap(uniq);
    }
    std::vector<DevLight> lights(d->n_lights);
    for (uint32_t i = 0; i < d->n_lights; ++i) {
        int li = d->lights[i];
        DevLight& L = lights[i];
        std::memset(&L, 0, sizeof(L));
        if (li < 0) {
            if (d->env_texture < 0) { g_err = "environment light without an env texture"; return RTG_ERR_ARG; }
            L.v1t.w = host_bits_f(1);
            continue;
        }
        if ((uint32_t)li >= nt) { g_err = "light triangle out of range"; return RTG_ERR_ARG; }
        const float* P = d->positions + (size_t)li * 9;
        const float* em = d->materials[d->material[li]].emission;
        L.v0a = make_float4(P[0], P[1], P[2], tri_area[li]);
        L.v1t = make_float4(P[3], P[4], P[5], host_bits_f(0));
        L.v2 = make_float4(P[6], P[7], P[8], 1.0f / tri_area[li]);  // Triangle::sample's pdf
        L.gn = make_float4(tri_gn[li * 3], tri_gn[li * 3 + 1], tri_gn[li * 3 + 2], 0.0f);
        L.em = make_float4(em[0], em[1], em[2], 0.0f);
    }
    if (d->camera.width < 1.0f || d->camera.height < 1.0f) { g_err = "bad film size"; return RTG_ERR_ARG; }
    hs.nodes = std::move(nodes);
    hs.nodesq = std::move(nodesq);
    hs.leafbox = std::move(leafbox);
    hs.tris48 = std::move(tris48);
    hs.shade = std::move(shade);
    hs.mats = std::move(mats);
    hs.lights = std::move(lights);
    hs.texinfo = std::move(texinfo);
    hs.texels = std::move(texels);
    hs.n_lights = (int)d->n_lights;
    hs.env_tex = d->env_texture;
    hs.env_off = d->env_texture >= 0 ? hs.texinfo[d->env_texture].off : 0;
    hs.env_w = d->env_texture >= 0 ? hs.texinfo[d->env_texture].w : 1;
    hs.env_h = d->env_texture >= 0 ? hs.texinfo[d->env_texture].h : 1;
    hs.env_uniform = d->env_texture >= 0 && uniform_tex[d->env_texture];
    for (int k = 0; k < 3; ++k) hs.env_one[k] = d->env_texture >= 0 ? d->textures[d->env_texture].texels[k] : 0.0f;
    hs.root_word = root_word;
    hs.root_wordw = root_wordw;
    for (int k = 0; k < 6; ++k) hs.root_box[k] = d->node_bounds[k];
    hs.cull_scale = scale;
    std::memcpy(hs.cam.ip, d->camera.inv_proj, sizeof(hs.cam.ip));
    std::memcpy(hs.cam.cm, d->camera.camera, sizeof(hs.cam.cm));
    hs.cam.ox = d->camera.origin[0];
    hs.cam.oy = d->camera.origin[1];
    hs.cam.oz = d->camera.origin[2];
    hs.cam.width = d->camera.width;
    hs.cam.height = d->camera.height;
    hs.proj = d->projection;
    return RTG_OK;
}

// The device half: upload the prepared records to `device`, allocate the film, size the launches.
int upload_scene(int device, const HostScene& hs, rtg_handle* h) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        g_err = "no HIP device available";
        return RTG_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= ndev) { g_err = "bad device index"; return RTG_ERR_ARG; }
    h->device = device;
    HIPOK(hipSetDevice(device));
    HIPOK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    hipDeviceProp_t prop;
    HIPOK(hipGetDeviceProperties(&prop, device));
    h->n_cu = prop.multiProcessorCount;
    h->bvh_depth = hs.bvh_depth;
    h->wide_depth = hs.wide_depth;
    h->rebuilt = hs.rebuilt;
    h->usew = hs.usew;
    int rc;
    if ((rc = dev_upload(&h->d_nodes, hs.nodes))) return rc;
    if ((rc = dev_upload(&h->d_nodesq, hs.nodesq))) return rc;
    if ((rc = dev_upload(&h->d_leafbox, hs.leafbox))) return rc;
    if (!hs.img.empty() && (rc = dev_upload(&h->d_img, hs.img))) return rc;
    if ((rc = dev_upload(&h->d_tris48, hs.tris48))) return rc;
    if ((rc = dev_upload(&h->d_shade, hs.shade))) return rc;
    if ((rc = dev_upload(&h->d_mats, hs.mats))) return rc;
    if ((rc = dev_upload(&h->d_lights, hs.lights))) return rc;
    if ((rc = dev_upload(&h->d_texinfo, hs.texinfo))) return rc;
    if ((rc = dev_upload(&h->d_texels, hs.texels))) return rc;

    SceneView& s = h->sv;
    s.nodes = h->d_nodes;
    s.tris48 = h->d_tris48;
    s.shade = h->d_shade;
    s.mats = h->d_mats;
    s.lights = h->d_lights;
    s.texinfo = h->d_texinfo;
    s.texels = (const float4*)h->d_texels;
    s.n_mats = (int)hs.mats.size();
    s.n_lights = hs.n_lights;
    s.pmf = 1.f / (float)hs.n_lights;  // Scene::sampleLight (Scene.h:137-138), the same IEEE division
    s.env_tex = hs.env_tex;
    s.env_off = hs.env_off;
    s.env_w = hs.env_w;
    s.env_h = hs.env_h;
    s.env_uniform = hs.env_uniform ? 1 : 0;
    for (int k = 0; k < 3; ++k) s.env_one[k] = hs.env_one[k];
    s.root_word = hs.root_word;
    s.nodesq = h->d_nodesq;
    s.leafbox = h->d_leafbox;
    s.root_wordw = hs.root_wordw;
    s.usew = hs.usew ? 1 : 0;
    s.img = hs.img.empty() ? nullptr : h->d_img;
    s.img_n4 = (int)hs.img.size();
    s.img_tri = hs.img_tri;
    s.img_lb = hs.img_lb;
    for (int k = 0; k < 6; ++k) s.root_box[k] = hs.root_box[k];
    s.cull_scale = hs.cull_scale;
    h->cam = hs.cam;
    h->proj = hs.proj;
    h->W = (int)hs.cam.width;
    h->H = (int)hs.cam.height;
    HIPOK(hipMalloc((void**)&h->d_film, (size_t)h->W * h->H * 3 * sizeof(float)));
    HIPOK(hipMemset(h->d_film, 0, (size_t)h->W * h->H * 3 * sizeof(float)));
    HIPOK(hipMalloc((void**)&h->d_qctr, 4 * sizeof(unsigned)));
    HIPOK(hipMalloc((void**)&h->d_stats, RTG_NSTATS * sizeof(unsigned long long)));
    HIPOK(hipMemset(h->d_stats, 0, RTG_NSTATS * sizeof(unsigned long long)));
    for (auto& e : h->ev) HIPOK(hipEventCreate(&e));

    int occ = 0;
    HIPOK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_trace<false, false>, RTG_TTB, 0));
    h->trace_blocks = h->n_cu * std::max(1, occ);
    HIPOK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_trace<true, false>, RTG_TTB, 0));
    h->trace_blocks_count = h->n_cu * std::max(1, occ);
    HIPOK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_trace<false, true>, RTG_TTB, 0));
    h->trace_blocks_small = h->n_cu * std::max(1, occ);
    HIPOK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_trace<true, true>, RTG_TTB, 0));
    h->trace_blocks_small_count = h->n_cu * std::max(1, occ);
    HIPOK(hipEventCreateWithFlags(&h->entry, hipEventDisableTiming));
    return ensure_ovf(h, h->slot[0]);
}

extern "C" {

int rtg_create(int device, const rtg_scene_desc* desc, rtg_handle** out) {
    if (!desc || !out) { g_err = "rtg_create: null argument"; return RTG_ERR_ARG; }
    rtg_handle* h = new rtg_handle();
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc == RTG_OK) rc = upload_scene(device, hs, h);
    if (rc != RTG_OK) {
        rtg_destroy(h);
        return rc;
    }
    *out = h;
    return RTG_OK;
}

void rtg_destroy(rtg_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    h->pend_n = 0;  // queued calls not issued yet are dropped with the film
    if (h->stream) {
        (void)join_frames(h);
        (void)hipStreamSynchronize(h->stream);
    }
    for (ChunkSlot& sl : h->slot) {
        free_chunk(sl);
        (void)hipFree(sl.d_ovf);
        if (sl.fold) (void)hipEventDestroy(sl.fold);
        if (sl.stream) (void)hipStreamDestroy(sl.stream);
    }
    if (h->entry) (void)hipEventDestroy(h->entry);
    (void)hipFree(h->d_img);
    (void)hipFree(h->d_nodes); (void)hipFree(h->d_nodesq); (void)hipFree(h->d_leafbox); (void)hipFree(h->d_tris48); (void)hipFree(h->d_shade); (void)hipFree(h->d_mats);
    (void)hipFree(h->d_lights); (void)hipFree(h->d_texinfo); (void)hipFree(h->d_texels); (void)hipFree(h->d_film);
    (void)hipFree(h->d_pix); (void)hipFree(h->d_qctr); (void)hipFree(h->d_stats);
    for (auto& e : h->ev) if (e) (void)hipEventDestroy(e);
    for (auto& e : h->kev) (void)hipEventDestroy(e);
    for (auto& e : h->tev) (void)hipEventDestroy(e);
    if (h->h_cnt) (void)hipHostFree(h->h_cnt);
    (void)hipFree(h->d_cap); (void)hipFree(h->d_cap_len); (void)hipFree(h->d_cap_rays);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int rtg_set_integrator(rtg_handle* h, int integrator) {
    if (!h || integrator < RTG_INTEGRATOR_PATH || integrator > RTG_INTEGRATOR_DIRECT_MIS) {
        g_err = "rtg_set_integrator: bad argument";
        return RTG_ERR_ARG;
    }
    if (int rc = flush_pending(h)) return rc;  // queued calls render with the settings they were queued under
    h->integrator = integrator;
    return RTG_OK;
}

int rtg_set_options(rtg_handle* h, int max_depth, int cull, uint32_t max_paths) {
    if (!h || max_depth < 0 || max_depth > 250) { g_err = "rtg_set_options: bad argument"; return RTG_ERR_ARG; }
    if (int rc = flush_pending(h)) return rc;  // queued calls render with the settings they were queued under
    h->max_depth = max_depth;
    h->cull = cull & 1;
    h->count = (cull >> 1) & 1;   // bit 1: counting kernels (node/triangle tests)
    h->timing = (cull >> 2) & 1;  // bit 2: per-launch timing events
    h->wide = ((cull >> 3) & 1) ? 0 : 1;  // bit 3: force the reference BVH2 walk
    h->wavetime = RTG_DEBUG ? (cull >> 4) & 1 : 0;  // bit 4 (RTG_DEBUG builds): per-wave clocks
    h->serial = (cull >> 5) & 1;  // bit 5: no frame pipeline, read-back k_shade grids
    h->no_coalesce = (cull >> 6) & 1;  // bit 6: queued calls are issued one by one
    if (max_paths) h->max_paths = max_paths;
    return RTG_OK;
}

}  // extern "C"

// Pixel list in tile order (32x32 tiles, row-major inside a tile), for the requested tiles.
int set_pixels(rtg_handle* h, const uint32_t* tiles, uint32_t n_tiles) {
    const int TS = 32;
    const uint32_t tx = (h->W + TS - 1) / TS, ty = (h->H + TS - 1) / TS;
    std::vector<uint32_t> key;
    if (tiles) key.assign(tiles, tiles + n_tiles);
    else key.push_back(0xffffffffu);
    if (h->d_pix && key == h->pix_key) return RTG_OK;
    std::vector<uint32_t> pix;
    auto add_tile = [&](uint32_t t) {
        uint32_t bx = (t % tx) * TS, by = (t / tx) * TS;
        for (uint32_t y = by; y < std::min<uint32_t>(by + TS, h->H); ++y)
            for (uint32_t x = bx; x < std::min<uint32_t>(bx + TS, h->W); ++x) pix.push_back(y * h->W + x);
    };
    if (tiles) {
        for (uint32_t i = 0; i < n_tiles; ++i) {
            if (tiles[i] >= tx * ty) { g_err = "tile id out of range"; return RTG_ERR_ARG; }
            add_tile(tiles[i]);
        }
    } else {
        for (uint32_t t = 0; t < tx * ty; ++t) add_tile(t);
    }
    // launches already queued may still read the old list (rtg_render_async, adaptive groups):
    // drain them before it is overwritten (hipMemcpy does not order against non-blocking streams)
    HIPOK(hipDeviceSynchronize());
    if (pix.size() > h->cap_pix) {
        (void)hipFree(h->d_pix);
        HIPOK(hipMalloc((void**)&h->d_pix, std::max<size_t>(pix.size(), 1) * 4));
        h->cap_pix = pix.size();
    }
    if (!pix.empty()) HIPOK(hipMemcpy(h->d_pix, pix.data(), pix.size() * 4, hipMemcpyHostToDevice));
    h->npix = (unsigned)pix.size();
    h->pix_key = key;
    return RTG_OK;
}

int launch_generate(rtg_handle* h, const ChunkArgs& a, const PathBufs& pb, hipStream_t st) {
    (void)h;
    hipLaunchKernelGGL(k_generate, dim3((a.P + RTG_TB - 1) / RTG_TB), dim3(RTG_TB), 0, st, a, pb);
    LAUNCH_OK("k_generate");
    return RTG_OK;
}

int launch_trace(rtg_handle* h, const TraceIO& io, hipStream_t st, unsigned max_blocks) {
    const bool small = h->sv.img != nullptr;
    auto g = [&](int full) { return dim3(max_blocks ? std::min<unsigned>((unsigned)full, max_blocks) : (unsigned)full); };
    if (h->count && small) hipLaunchKernelGGL((k_trace<true, true>), g(h->trace_blocks_small_count), dim3(RTG_TTB), 0, st, h->sv, io);
    else if (h->count) hipLaunchKernelGGL((k_trace<true, false>), g(h->trace_blocks_count), dim3(RTG_TTB), 0, st, h->sv, io);
    else if (small) hipLaunchKernelGGL((k_trace<false, true>), g(h->trace_blocks_small), dim3(RTG_TTB), 0, st, h->sv, io);
    else hipLaunchKernelGGL((k_trace<false, false>), g(h->trace_blocks), dim3(RTG_TTB), 0, st, h->sv, io);
    LAUNCH_OK("k_trace");
    return RTG_OK;
}

static void timed_begin(rtg_handle* h, hipStream_t st, size_t k) {
    if (!h->timing) return;
    while (h->kev.size() < 2 * (k + 1)) { hipEvent_t e; (void)hipEventCreate(&e); h->kev.push_back(e); }
    (void)hipEventRecord(h->kev[2 * k], st);
}
static void timed_end(rtg_handle* h, hipStream_t st, size_t k) {
    if (h->timing) (void)hipEventRecord(h->kev[2 * k + 1], st);
}

// RTG_DEBUG builds, RTG_OPT_WAVETIME: per launch, when the waves started, found the queue empty and ended
static void print_wavetime(const std::vector<unsigned long long>& wt, int maxb, size_t wt_waves) {
    for (int b = 0; b <= maxb; ++b) {
        const unsigned long long* w = wt.data() + (size_t)b * wt_waves * 3;
        unsigned long long t0 = ~0ull, e0 = ~0ull;
        std::vector<double> ends, starts;
        for (size_t i = 0; i < wt_waves; ++i) {
            if (!w[3 * i]) continue;
            t0 = std::min(t0, w[3 * i]);
            if (w[3 * i + 1]) e0 = std::min(e0, w[3 * i + 1]);
        }
        for (size_t i = 0; i < wt_waves; ++i) {
            if (!w[3 * i]) continue;
            starts.push_back((w[3 * i] - t0) * 0.01);  // 100 MHz clock -> us
            ends.push_back((w[3 * i + 2] - t0) * 0.01);
        }
        if (ends.empty()) continue;
        std::sort(ends.begin(), ends.end());
        std::sort(starts.begin(), starts.end());
        auto pct = [](const std::vector<double>& v, double q) { return v[std::min(v.size() - 1, (size_t)(q * v.size()))]; };
        std::fprintf(stderr, "[wavetime] launch %d waves %zu start p50 %.1f max %.1f | queue empty %.1f | "
                     "wave end p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f us\n", b, ends.size(), pct(starts, 0.5),
                     starts.back(), (e0 - t0) * 0.01, pct(ends, 0.1), pct(ends, 0.5), pct(ends, 0.9), pct(ends, 0.99),
                     ends.back());
    }
}

const char* roctx_stage_name(int kind, int b) {
    static const char* const trace[32] = {
        "rtg:trace b=0", "rtg:trace b=1", "rtg:trace b=2", "rtg:trace b=3", "rtg:trace b=4", "rtg:trace b=5",
        "rtg:trace b=6", "rtg:trace b=7", "rtg:trace b=8", "rtg:trace b=9", "rtg:trace b=10", "rtg:trace b=11",
        "rtg:trace b=12", "rtg:trace b=13", "rtg:trace b=14", "rtg:trace b=15", "rtg:trace b=16", "rtg:trace b=17",
        "rtg:trace b=18", "rtg:trace b=19", "rtg:trace b=20", "rtg:trace b=21", "rtg:trace b=22", "rtg:trace b=23",
        "rtg:trace b=24", "rtg:trace b=25", "rtg:trace b=26", "rtg:trace b=27", "rtg:trace b=28", "rtg:trace b=29",
        "rtg:trace b=30", "rtg:trace b=31"};
    static const char* const shade[32] = {
        "rtg:shade b=0", "rtg:shade b=1", "rtg:shade b=2", "rtg:shade b=3", "rtg:shade b=4", "rtg:shade b=5",
        "rtg:shade b=6", "rtg:shade b=7", "rtg:shade b=8", "rtg:shade b=9", "rtg:shade b=10", "rtg:shade b=11",
        "rtg:shade b=12", "rtg:shade b=13", "rtg:shade b=14", "rtg:shade b=15", "rtg:shade b=16", "rtg:shade b=17",
        "rtg:shade b=18", "rtg:shade b=19", "rtg:shade b=20", "rtg:shade b=21", "rtg:shade b=22", "rtg:shade b=23",
        "rtg:shade b=24", "rtg:shade b=25", "rtg:shade b=26", "rtg:shade b=27", "rtg:shade b=28", "rtg:shade b=29",
        "rtg:shade b=30", "rtg:shade b=31"};
    if (b < 0 || b >= 32) return kind ? "rtg:shade" : "rtg:trace";
    return kind ? shade[b] : trace[b];
}

// The 8 segment counts of bounce b that k_trace(b)'s block 0 stores into h_cnt as it starts. The
// host polls the host-coherent words; a launch that ended (or failed) without writing them is an
// error, not a hang.
static int wait_counts(rtg_handle* h, int b) {
    unsigned* c = h->h_cnt + 8 * b;
    auto ready = [&]() {
        for (int k = 0; k < 8; ++k)
            if (__atomic_load_n(c + k, __ATOMIC_ACQUIRE) == RTG_CNT_PENDING) return false;
        return true;
    };
    for (unsigned spin = 1;; ++spin) {
        if (ready()) return RTG_OK;
        if ((spin & 255u) == 0) {
            const hipError_t e = hipEventQuery(h->tev[b]);
            if (e == hipSuccess) {
                if (ready()) return RTG_OK;
                g_err = "k_trace finished without storing its segment counts";
                return RTG_ERR_HIP;
            }
            if (e != hipErrorNotReady) {
                g_err = std::string("k_trace (segment counts): ") + hipGetErrorString(e);
                return RTG_ERR_HIP;
            }
            std::this_thread::yield();
        }
    }
}

int render_impl(rtg_handle* h, uint32_t first, uint32_t n_samples, uint64_t seed,
                       const uint32_t* tiles, uint32_t n_tiles, hipStream_t st, bool lazy, bool add_spp) {
    RoctxRange r_render(lazy ? "rtg:render (queued chunks)" : "rtg:render");
    int rc = set_pixels(h, tiles, n_tiles);
    if (rc) return rc;
    if (h->npix == 0 || n_samples == 0) return RTG_OK;
    if ((uint64_t)first + n_samples > 65536u) { g_err = "sample index >= 65536 (PCG stream key)"; return RTG_ERR_ARG; }
    const int maxb = h->max_depth + 2;
    // computeDirectMIS keeps two scratch planes of per-path state in contrib planes 2 and 3
    const int planes = h->integrator == RTG_INTEGRATOR_DIRECT_MIS ? std::max(maxb, 4) : maxb;
    uint32_t ns_chunk = std::max<uint32_t>(1, std::min<uint32_t>(n_samples, h->max_paths / std::max(1u, h->npix)));
    // the diagnostic modes read one chunk's launches in order on one stream (per-launch timing
    // events work across the slots' streams: overlapped launches then count their shared time twice)
    const bool diag = h->serial || (RTG_DEBUG && (h->wavetime || h->capture_launch >= 0));
    {
        // path state of the chunks in flight takes at most RTG_MEM_PCT % of the free HBM (buffers held
        // now count as free); pipelined chunks keep RTG_SLOTS sets
        size_t freeb = 0, totalb = 0;
        if (hipMemGetInfo(&freeb, &totalb) == hipSuccess) {
            size_t held = 0;
            for (const ChunkSlot& sl : h->slot) held += slot_bytes(sl);
            size_t budget = (freeb + held) / 100 * RTG_MEM_PCT;
            if (h->mem_cap) budget = std::min(budget, h->mem_cap);
            const size_t per_pix = path_bytes(planes, false) * std::max<size_t>(1, h->npix);
            size_t max_ns = budget / per_pix;
            if (lazy && !diag && (size_t)ns_chunk * h->npix <= RTG_PIPE_MAX_P) max_ns = budget / RTG_SLOTS / per_pix;
            ns_chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(ns_chunk, max_ns));
        }
    }
    // Keep the chunk buffers once they hold most of what the budget asks for: the free-memory
    // reading moves between calls, and growing a buffer of ~100 GB means a free and a new
    // hipMalloc that took 5.5 s on C4 with 1G paths in flight.
    {
        const ChunkSlot& s0 = h->slot[0];
        const uint32_t fit = s0.cap_maxb >= planes ? (uint32_t)(s0.cap_P / std::max(1u, h->npix)) : 0u;
        if (fit >= 1 && ns_chunk > fit && (uint64_t)fit * 4 >= (uint64_t)ns_chunk * 3) ns_chunk = fit;
    }
    // equal chunks: 256 samples at <= 123 per chunk run as 86 + 85 + 85, not 123 + 123 + 10 (a thin
    // last chunk is mostly drain tail)
    {
        const uint32_t nchunks = (n_samples + ns_chunk - 1) / ns_chunk;
        ns_chunk = (n_samples + nchunks - 1) / nchunks;
    }
    const size_t P = (size_t)ns_chunk * h->npix;
    h->stats.chunk_samples = std::max<uint64_t>(h->stats.chunk_samples, ns_chunk);
    // the frame pipeline (rtg_internal.h, ChunkSlot): queued chunks of up to RTG_PIPE_MAX_P paths
    // rotate through the slots with no host wait, so the next queued frames run beside them. A call
    // that is waited for runs its chunks one at a time in slot 0: chunks of one render side by side
    // measured slower than one chunk (C3 at N = 1 and rank 0's share of 8: the traversals slow each
    // other down and add launches)
    const bool pipe = lazy && !diag && P <= RTG_PIPE_MAX_P;
    (void)hipGetLastError();  // drop any stale error left by other code on this thread
    if (!h->inflight) HIPOK(hipEventRecord(h->ev[0], st));  // start of this render (or of a queued run)
    HIPOK(hipEventRecord(h->entry, st));  // every chunk starts after the caller's earlier work on st
    std::vector<int> kinds;  // 0 trace, 2 other (timing mode)
    size_t k = 0;
    TraceIO io{};
    io.stats = h->d_stats;
    io.cull = h->cull;
    io.wide = h->wide;
    // RTG_DEBUG builds with RTG_OPT_WAVETIME: per-wave clocks of chunk 0's trace launches, on stderr
    unsigned long long* d_wt = nullptr;
    const size_t wt_waves = (size_t)std::max(std::max(h->trace_blocks, h->trace_blocks_count),
                                             std::max(h->trace_blocks_small, h->trace_blocks_small_count)) * (RTG_TTB / 64);
    if (h->cap_cnt < maxb + 1) {
        if (h->h_cnt) (void)hipHostFree(h->h_cnt);
        h->h_cnt = h->d_hcnt = nullptr;
        h->cap_cnt = 0;
        HIPOK(hipHostMalloc((void**)&h->h_cnt, (size_t)(maxb + 1) * 8 * sizeof(unsigned),
                            hipHostMallocCoherent | hipHostMallocMapped));
        HIPOK(hipHostGetDevicePointer((void**)&h->d_hcnt, h->h_cnt, 0));
        h->cap_cnt = maxb + 1;
    }
    while ((int)h->tev.size() < maxb + 1) {
        hipEvent_t e;
        HIPOK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        h->tev.push_back(e);
    }
    uint32_t c = 0;
    for (uint32_t s0 = first; s0 < first + n_samples; s0 += ns_chunk, ++c) {
        ChunkSlot& sl = pipe ? h->slot[h->next_slot++ % RTG_SLOTS] : h->slot[0];
        // back-pressure: a slot takes its next chunk once its previous one has left the GPU, so at
        // most RTG_SLOTS chunks are in flight and the host stays at most that far ahead
        if (pipe && sl.used) HIPOK(hipEventSynchronize(sl.fold));
        if ((rc = ensure_chunk(h, sl, P, planes, false))) return rc;
        if ((rc = ensure_ovf(h, sl))) return rc;
        const hipStream_t ss = sl.stream;
        PathBufs& pb = sl.pb;
        io.ovf = sl.d_ovf;
        // A chunk starts after the caller's earlier work on st. A queued (pipelined) chunk reads
        // nothing the caller's work on the handle's stream writes (film reads and gathers, film
        // loads; pixel lists and clears wait for the device on the host), so only its fold waits
        // for that work, below: the chunk's traversal can start while earlier frames drain.
        if (!pipe) HIPOK(hipStreamWaitEvent(ss, h->entry, 0));
        if (RTG_DEBUG && h->wavetime && c == 0) {
            HIPOK(hipMalloc((void**)&d_wt, (size_t)(maxb + 1) * wt_waves * 3 * sizeof(unsigned long long)));
            HIPOK(hipMemsetAsync(d_wt, 0, (size_t)(maxb + 1) * wt_waves * 3 * sizeof(unsigned long long), ss));
        }
        ChunkArgs a;
        a.pixlist = h->d_pix;
        a.npix = h->npix;
        a.ns = std::min(ns_chunk, first + n_samples - s0);
        a.s0 = s0;
        a.P = a.ns * h->npix;
        a.seed = seed;
        a.max_depth = h->max_depth;
        a.mode = h->integrator;
        a.cam = h->cam;
        a.lean = 1;
        a.seg_tiles = (unsigned)seg_tiles(a.P);
        set_ns_div(a);
        // k_shade grids from the live counts read back while the traversal runs (big chunks), or over
        // every tile a segment can hold (blocks past the live count exit at once): no host wait
        const bool hostgrid = !pipe && (a.seg_tiles >= RTG_HOSTGRID_MIN_TILES || h->serial);
        HIPOK(hipMemsetAsync(pb.ctr, 0, (size_t)(maxb + 1) * sizeof(Counters), ss));
        timed_begin(h, ss, k);
        {
            RoctxRange r_gen("rtg:generate");
            hipLaunchKernelGGL(k_generate, dim3((a.npix + RTG_TB - 1) / RTG_TB), dim3(RTG_TB), 0, ss, a, pb);  // lean: per pixel
            LAUNCH_OK("k_generate");
        }
        timed_end(h, ss, k); kinds.push_back(2); ++k;
        // Trace launch L_b (b = 0..maxb) carries the extension rays of bounce b (from shade(b-1),
        // or generate) and the shadow rays of bounce b-1: one persistent launch, one drain tail.
        for (int b = 0; b <= maxb; ++b) {
            if (b > 0) {
                RoctxRange r_shade(roctx_stage_name(1, b - 1));
                // one 256-path tile per block: 8 x the largest segment's live tiles (the segment
                // counts of bounce b - 1 arrived while k_trace(b - 1) ran; bounce 0: the camera rays)
                unsigned tiles = hostgrid ? 0u : a.seg_tiles;
                const unsigned cap = a.seg_tiles * RTG_TB;
                for (int sgm = 0; hostgrid && sgm < 8; ++sgm) {
                    unsigned live = 0;
                    if (b == 1) {
                        live = a.P > sgm * cap ? std::min(cap, a.P - sgm * cap) : 0u;
                    } else {
                        if (sgm == 0 && (rc = wait_counts(h, b - 1))) return rc;
                        live = h->h_cnt[8 * (b - 1) + sgm];
                    }
                    tiles = std::max(tiles, (live + RTG_TB - 1) / RTG_TB);
                }
                if (tiles) {
                    timed_begin(h, ss, k);
                    const bool tab = h->sv.n_mats <= RTG_LDS_MATS && h->sv.n_lights <= RTG_LDS_LIGHTS;
                    const bool alt = h->integrator != RTG_INTEGRATOR_PATH;
                    if (int rc_ = launch_shade(alt, tab, 8 * tiles, ss, h->sv, a, pb, b - 1)) return rc_;
                    timed_end(h, ss, k); kinds.push_back(2); ++k;
                }
            }
            // extension payload by queue position (set b & 1; null queue: path id = position);
            // bounce 0: the camera origin, directions from k_generate in set 0
            io.queue = nullptr;
            io.ray_o = b == 0 ? nullptr : ((b & 1) ? pb.ray_o2 : pb.ray_o);
            io.cam_o = make_float4(a.cam.ox, a.cam.oy, a.cam.oz, 0.0f);
            io.ray_d = (b & 1) ? pb.ray_d2 : pb.ray_d;
            // segmented queues; bounce 0: one queue of npix camera rays (a ray per pixel, shared by
            // the pixel's samples) at identity positions, one work counter
            io.count = b == 0 ? &pb.ctr[0].n_cam : nullptr;
            io.seg_cap = b == 0 ? 0u : a.seg_tiles * RTG_TB;
            io.seg_ne = (b > 0 && b < maxb) ? pb.ctr[b].ne8 : nullptr;
            io.seg_ns = b > 0 ? pb.ctr[b - 1].ns8 : nullptr;
            io.hits = pb.hits;
            io.squeue = pb.shq;
            io.sray_o = pb.sh_o;
            io.sray_d = pb.sh_d;
            io.sray_c = pb.sh_c;
            io.spos = 1;
            io.scount = nullptr;
            io.contrib = b > 0 ? pb.contrib + (size_t)(b - 1) * a.P : nullptr;
            io.visible = nullptr;
            io.fetch = &pb.ctr[b].f_ext;
            io.fetch8 = b == 0 ? nullptr : pb.ctr[b].f8;
            io.wtime = (d_wt && c == 0) ? d_wt + (size_t)b * wt_waves * 3 : nullptr;
            io.cap = nullptr;
            io.cap_len = nullptr;
            // k_trace(b) hands the host bounce b's segment counts, for k_shade(b)'s grid
            io.hcnt = nullptr;
            if (hostgrid && b > 0 && b < maxb) {
                for (int k = 0; k < 8; ++k) __atomic_store_n(h->h_cnt + 8 * b + k, RTG_CNT_PENDING, __ATOMIC_RELAXED);
                io.hcnt = h->d_hcnt + 8 * b;
            }
            if (RTG_DEBUG && c == 0 && b == h->capture_launch) {
                const size_t cn = 2 * (size_t)a.seg_tiles * 8 * RTG_TB;  // both index spans
                (void)hipFree(h->d_cap);
                (void)hipFree(h->d_cap_len);
                h->d_cap = nullptr;
                h->d_cap_len = nullptr;
                HIPOK(hipMalloc((void**)&h->d_cap, cn * (RTG_CAP_LEN / 4) * sizeof(uint4)));
                HIPOK(hipMalloc((void**)&h->d_cap_len, cn * sizeof(unsigned)));
                if (!h->d_cap_rays) HIPOK(hipMalloc((void**)&h->d_cap_rays, 35 * sizeof(unsigned)));
                HIPOK(hipMemsetAsync(h->d_cap_len, 0, cn * sizeof(unsigned), ss));
                hipLaunchKernelGGL(k_cap_slices, dim3(1), dim3(64), 0, ss, io, h->d_cap_rays);
                LAUNCH_OK("k_cap_slices");
                h->cap_n = (unsigned)cn;
                io.cap = h->d_cap;
                io.cap_len = h->d_cap_len;
                io.cap_n = (unsigned)cn;
            }
            timed_begin(h, ss, k);
            {
                RoctxRange r_trace(roctx_stage_name(0, b));
                // the camera launch (a ray per pixel, one work counter): with RTG_CAM_GRID, no more
                // one-wave blocks than it has tail batches of rays, so waves without work do not
                // queue their probes on the counter
                const unsigned cam_blocks = (RTG_CAM_GRID && b == 0)
                                                ? std::max(8u, (a.npix + RTG_TAIL_BATCH - 1) / RTG_TAIL_BATCH) : 0u;
                if ((rc = launch_trace(h, io, ss, cam_blocks))) return rc;
            }
            timed_end(h, ss, k); kinds.push_back(0); ++k;
            if (io.hcnt) HIPOK(hipEventRecord(h->tev[b], ss));
        }
        hipLaunchKernelGGL(k_tally, dim3(1), dim3(64), 0, ss, pb.ctr, maxb, h->d_stats);
        LAUNCH_OK("k_tally");
        // the film takes the chunks in sample order: this fold runs after the previous chunk's
        RoctxRange r_acc("rtg:accumulate");
        if (h->last_fold) HIPOK(hipStreamWaitEvent(ss, h->last_fold, 0));
        if (pipe) HIPOK(hipStreamWaitEvent(ss, h->entry, 0));  // the film's readers and writers so far
        timed_begin(h, ss, k);
        if (a.ns > 1) {
            const unsigned ppw = a.ns <= 32 ? 64u / (a.ns < 4 ? 4u : a.ns) : 1u;  // pixels per wave (k_accumulate_pm)
            const unsigned waves = (h->npix + ppw - 1) / ppw;
            hipLaunchKernelGGL(k_accumulate_pm, dim3((waves + RTG_TB / 64 - 1) / (RTG_TB / 64)), dim3(RTG_TB), 0, ss, a,
                               pb, h->d_film);
        } else
            hipLaunchKernelGGL(k_accumulate, dim3((h->npix + RTG_TB - 1) / RTG_TB), dim3(RTG_TB), 0, ss, a, pb, h->d_film);
        LAUNCH_OK("k_accumulate");
        timed_end(h, ss, k); kinds.push_back(2); ++k;
        HIPOK(hipEventRecord(sl.fold, ss));
        sl.used = true;
        h->last_fold = sl.fold;
        h->inflight = true;
        h->stats.paths += a.P;
        if (d_wt) {
            std::vector<unsigned long long> wt((size_t)(maxb + 1) * wt_waves * 3);
            HIPOK(hipStreamSynchronize(ss));
            HIPOK(hipMemcpy(wt.data(), d_wt, wt.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            (void)hipFree(d_wt);
            d_wt = nullptr;
            print_wavetime(wt, maxb, wt_waves);
        }
    }
    if (add_spp) h->spp += n_samples;
    if (lazy) return RTG_OK;
    // the caller's stream waits for the chunks (and for every chunk queued before them). The queued
    // chunks are joined to the handle's own stream only when that is the caller's stream; a render
    // on a user stream leaves them in flight, so join_frames (film read, clear, stats) still makes
    // the handle's stream wait for them
    if (st == h->stream) h->inflight = false;
    HIPOK(hipStreamWaitEvent(st, h->last_fold, 0));
    HIPOK(hipEventRecord(h->ev[1], st));
    if (h->timing) {
        HIPOK(hipEventSynchronize(h->ev[1]));
        h->stats.extend_ms = h->stats.shadow_ms = h->stats.shade_ms = 0;
        h->stats.extend_launches = 0;
        h->launch_ms.clear();
        // the rays of each trace launch of the last chunk (camera rays, then extension + shadow rays)
        h->launch_rays.clear();
        std::vector<Counters> cc((size_t)maxb + 1);
        // (a waited-for render runs its chunks in slot 0)
        if (h->slot[0].pb.ctr &&
            hipMemcpy(cc.data(), h->slot[0].pb.ctr, cc.size() * sizeof(Counters), hipMemcpyDeviceToHost) == hipSuccess) {
            for (int b = 0; b <= maxb; ++b) {
                unsigned long long r = b == 0 ? cc[0].n_cam : 0ull;
                for (int k = 0; k < 8; ++k) {
                    if (b > 0 && b < maxb) r += cc[b].ne8[32 * k];
                    if (b > 0) r += cc[b - 1].ns8[32 * k];
                }
                h->launch_rays.push_back(r);
            }
        }
        for (size_t j = 0; j < kinds.size(); ++j) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, h->kev[2 * j], h->kev[2 * j + 1]);
            (kinds[j] == 0 ? h->stats.extend_ms : h->stats.shade_ms) += ms;
            if (kinds[j] == 0) {
                h->stats.extend_launches++;
                h->launch_ms.push_back(ms);
            }
        }
    }
    return RTG_OK;
}

extern "C" {

int rtg_render_async(rtg_handle* h, uint32_t first, uint32_t n, uint64_t seed, const uint32_t* tiles,
                     uint32_t n_tiles, void* stream) {
    if (!h) { g_err = "null handle"; return RTG_ERR_ARG; }
    HIPOK(hipSetDevice(h->device));
    if (stream) {
        if (int rc = flush_pending(h)) return rc;
        return render_impl(h, first, n, seed, tiles, n_tiles, (hipStream_t)stream, false);
    }
    if (n == 0) return RTG_OK;
    if ((uint64_t)first + n > 65536u) { g_err = "sample index >= 65536 (PCG stream key)"; return RTG_ERR_ARG; }
    // queued: coalesced with the pending calls when it continues them (same seed and tiles, the
    // next sample indices); otherwise those are issued first
    std::vector<uint32_t> key;
    if (tiles) key.assign(tiles, tiles + n_tiles);
    else key.push_back(0xffffffffu);
    if (h->pend_n && (key != h->pend_key || seed != h->pend_seed || first != h->pend_first + h->pend_n))
        if (int rc = flush_pending(h)) return rc;
    if (int rc = set_pixels(h, tiles, n_tiles)) return rc;  // (validates the tiles; a no-op when unchanged)
    if (!h->pend_n) {
        h->pend_first = first;
        h->pend_seed = seed;
        h->pend_key.swap(key);
    }
    if (h->npix == 0) return RTG_OK;  // no pixels: nothing is rendered and Film::SPP stays (as rtg_render)
    h->pend_n += n;
    h->spp += n;  // Film::SPP counts the queued frames at once (taken back if their issue fails)
    if (h->no_coalesce || (uint64_t)h->pend_n * h->npix >= RTG_COALESCE_P) return flush_pending(h);
    return RTG_OK;
}

int rtg_render(rtg_handle* h, uint32_t first, uint32_t n, uint64_t seed, const uint32_t* tiles, uint32_t n_tiles) {
    if (!h) { g_err = "null handle"; return RTG_ERR_ARG; }
    HIPOK(hipSetDevice(h->device));
    if (int rc = flush_pending(h)) return rc;
    int rc = render_impl(h, first, n, seed, tiles, n_tiles, h->stream, false);
    if (rc) return rc;
    return rtg_synchronize(h);
}

int rtg_render_idle(rtg_handle* h, int* idle) {
    if (!h || !idle) { g_err = "rtg_render_idle: null argument"; return RTG_ERR_ARG; }
    HIPOK(hipSetDevice(h->device));
    if (int rc = flush_pending(h)) return rc;  // queued calls not issued yet are work left
    *idle = 1;
    if (h->last_fold) {
        const hipError_t e = hipEventQuery(h->last_fold);
        if (e == hipErrorNotReady) *idle = 0;
        else if (e != hipSuccess) { g_err = std::string("rtg_render_idle: ") + hipGetErrorString(e); return RTG_ERR_HIP; }
    }
    if (*idle) {
        const hipError_t e = hipStreamQuery(h->stream);
        if (e == hipErrorNotReady) *idle = 0;
        else if (e != hipSuccess) { g_err = std::string("rtg_render_idle: ") + hipGetErrorString(e); return RTG_ERR_HIP; }
    }
    return RTG_OK;
}

int rtg_render_adaptive(rtg_handle* h, uint32_t first, uint64_t seed, uint32_t init_samples, uint32_t max_samples,
                        uint32_t min_samples, uint32_t* tile_samples) {
    if (!h || init_samples == 0) { g_err = "rtg_render_adaptive: bad argument"; return RTG_ERR_ARG; }
    HIPOK(hipSetDevice(h->device));
    if (int rc0 = join_frames(h)) return rc0;
    hipStream_t st = h->stream;
    const size_t nf = (size_t)h->W * h->H * 3;
    const uint32_t spp0 = h->spp;
    const int TS = 32;
    const uint32_t tx = (h->W + TS - 1) / TS, ty = (h->H + TS - 1) / TS, nt = tx * ty;
    float* d_tmp = nullptr;
    HIPOK(hipMalloc((void**)&d_tmp, nf * sizeof(float)));
    float* d_keep = h->d_film;
    auto fail = [&](int rc) { h->d_film = d_keep; (void)hipFree(d_tmp); h->spp = spp0; return rc; };
    // ---- pass 1 (adaptiveSampling, Renderer.h:583-638): per-pixel sums of init_samples samples
    h->d_film = d_tmp;
    if (hipMemsetAsync(d_tmp, 0, nf * sizeof(float), st) != hipSuccess) return fail(RTG_ERR_HIP);
    int rc = render_impl(h, first, init_samples, seed, nullptr, 0, st, false);
    if (rc) return fail(rc);
    std::vector<float> sums(nf);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(sums.data(), d_tmp, nf * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) {
        g_err = "rtg_render_adaptive: pass-1 readback failed";
        return fail(RTG_ERR_HIP);
    }
    std::vector<float> var(nt, 0.0f);
    const float fi = (float)init_samples;
    std::vector<float> est;
    for (uint32_t t = 0; t < nt; ++t) {
        const uint32_t x0 = (t % tx) * TS, y0 = (t / tx) * TS;
        const uint32_t x1 = std::min<uint32_t>(x0 + TS, h->W), y1 = std::min<uint32_t>(y0 + TS, h->H);
        est.clear();
        for (uint32_t y = y0; y < y1; ++y)
            for (uint32_t x = x0; x < x1; ++x)
                for (int c = 0; c < 3; ++c) est.push_back(sums[((size_t)y * h->W + x) * 3 + c] / fi);
        const int n = (int)(est.size() / 3);
        float gt[3] = {0.0f, 0.0f, 0.0f}, sq[3] = {0.0f, 0.0f, 0.0f};
        for (int i = 0; i < n; ++i)
            for (int c = 0; c < 3; ++c) gt[c] = gt[c] + est[3 * i + c];
        for (int c = 0; c < 3; ++c) gt[c] = gt[c] / (float)n;
        for (int i = 0; i < n; ++i)
            for (int c = 0; c < 3; ++c) {
                const float d = est[3 * i + c] - gt[c];
                sq[c] = sq[c] + d * d;
            }
        var[t] = (((sq[0] + sq[1]) + sq[2]) / 3.0f) / (float)(n - 1);
    }
    float total = 0.0f;
    for (uint32_t t = 0; t < nt; ++t) total += var[t];
    // ---- pass 2 (sampleTileWithWeight, Renderer.h:640-672): tiles grouped by sample count
    std::vector<std::pair<uint32_t, uint32_t>> cnt(nt);  // (samples, tile)
    for (uint32_t t = 0; t < nt; ++t) {
        float w = (total > 0.0f) ? var[t] / total : 0.0f;
        w = std::sqrt(w);
        int smp = (int)(w * (float)max_samples);
        smp = smp > (int)min_samples ? smp : (int)min_samples;
        cnt[t] = {(uint32_t)smp, t};
        if (tile_samples) tile_samples[t] = (uint32_t)smp;
    }
    std::sort(cnt.begin(), cnt.end());
    // every pass-2 sample index must stay inside the PCG key (seq = pixel << 16 | sample): checked
    // before the film is touched
    if (!cnt.empty() && (uint64_t)first + init_samples + cnt.back().first > RTG_MAX_SAMPLES_PER_KEY) {
        g_err = "rtg_render_adaptive: first_sample + init_samples + max tile count exceeds 65536";
        return fail(RTG_ERR_ARG);
    }
    // pass 2 folds into a staged copy of the film, published only when every group succeeded
    float* d_acc = nullptr;
    if (hipMalloc((void**)&d_acc, nf * sizeof(float)) != hipSuccess) { g_err = "rtg_render_adaptive: out of memory"; return fail(RTG_ERR_HIP); }
    auto fail2 = [&](int rc) { (void)hipFree(d_acc); return fail(rc); };
    if (hipMemcpyAsync(d_acc, d_keep, nf * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess) return fail2(RTG_ERR_HIP);
    for (size_t i = 0; i < cnt.size();) {
        size_t j = i;
        std::vector<uint32_t> group;
        while (j < cnt.size() && cnt[j].first == cnt[i].first) group.push_back(cnt[j++].second);
        const uint32_t n = cnt[i].first;
        i = j;
        if (n == 0) continue;
        h->d_film = d_tmp;
        if (hipMemsetAsync(d_tmp, 0, nf * sizeof(float), st) != hipSuccess) return fail2(RTG_ERR_HIP);
        if ((rc = render_impl(h, first + init_samples, n, seed, group.data(), (uint32_t)group.size(), st, false))) return fail2(rc);
        h->d_film = d_keep;
        hipLaunchKernelGGL(k_fold_mean, dim3((h->npix + RTG_TB - 1) / RTG_TB), dim3(RTG_TB), 0, st, h->d_pix, h->npix,
                           (const float*)d_tmp, (float)n, d_acc);
        if (hipGetLastError() != hipSuccess) { g_err = "launch k_fold_mean failed"; return fail2(RTG_ERR_HIP); }
    }
    h->d_film = d_keep;
    if (hipMemcpyAsync(d_keep, d_acc, nf * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess) return fail2(RTG_ERR_HIP);
    HIPOK(hipStreamSynchronize(st));
    (void)hipFree(d_acc);
    (void)hipFree(d_tmp);
    h->spp = spp0 + 1;  // render(): film->incrementSPP() once per frame
    return RTG_OK;
}

int rtg_launch_times(rtg_handle* h, double* trace_ms, uint32_t max, uint32_t* n) {
    if (!h || !n) return RTG_ERR_ARG;
    *n = (uint32_t)h->launch_ms.size();
    for (uint32_t i = 0; trace_ms && i < std::min<uint32_t>(max, *n); ++i) trace_ms[i] = h->launch_ms[i];
    return RTG_OK;
}

int rtg_launch_rays(rtg_handle* h, uint64_t* rays, uint32_t max, uint32_t* n) {
    if (!h || !n) return RTG_ERR_ARG;
    *n = (uint32_t)h->launch_rays.size();
    for (uint32_t i = 0; rays && i < std::min<uint32_t>(max, *n); ++i) rays[i] = h->launch_rays[i];
    return RTG_OK;
}

int rtg_debug_capture(rtg_handle* h, int launch) {
    if (!h) return RTG_ERR_ARG;
    if (!RTG_DEBUG) { g_err = "rtg_debug_capture: diagnostic builds only (RTG_DEBUG=1)"; return RTG_ERR_ARG; }
    h->capture_launch = launch;
    return RTG_OK;
}

int rtg_debug_replay(rtg_handle* h, double* out) {
    if (!h || !out) return RTG_ERR_ARG;
#if RTG_DEBUG
    if (!h->d_cap) { g_err = "rtg_debug_replay: nothing captured"; return RTG_ERR_ARG; }
    HIPOK(hipSetDevice(h->device));
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipStreamSynchronize(h->stream));
    unsigned tab[35];
    HIPOK(hipMemcpy(tab, h->d_cap_rays, sizeof(tab), hipMemcpyDeviceToHost));
    const unsigned rays[2] = {tab[33], tab[34]};
    unsigned* d_f8 = nullptr;
    unsigned long long* d_tot = nullptr;
    float* d_out = nullptr;
    HIPOK(hipMalloc((void**)&d_f8, 8 * 32 * sizeof(unsigned)));
    HIPOK(hipMalloc((void**)&d_tot, sizeof(unsigned long long)));
    HIPOK(hipMalloc((void**)&d_out, sizeof(float)));
    hipEvent_t e0, e1;
    HIPOK(hipEventCreate(&e0));
    HIPOK(hipEventCreate(&e1));
    float best = 1e30f;
    unsigned long long tot = 0;
    for (int rep = 0; rep < 3; ++rep) {
        HIPOK(hipMemsetAsync(d_f8, 0, 8 * 32 * sizeof(unsigned), h->stream));
        HIPOK(hipMemsetAsync(d_tot, 0, sizeof(unsigned long long), h->stream));
        HIPOK(hipEventRecord(e0, h->stream));
        hipLaunchKernelGGL(k_replay, dim3(std::max(1, h->trace_blocks * RTG_TTB / RTG_TB)), dim3(RTG_TB), 0, h->stream, h->sv, (const uint4*)h->d_cap,
                           (const unsigned*)h->d_cap_len, (const unsigned*)h->d_cap_rays, h->cap_n, 0u, d_f8, d_tot,
                           d_out);
        LAUNCH_OK("k_replay");
        HIPOK(hipEventRecord(e1, h->stream));
        HIPOK(hipEventSynchronize(e1));
        float ms = 0;
        HIPOK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
        HIPOK(hipMemcpy(&tot, d_tot, sizeof(tot), hipMemcpyDeviceToHost));
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(d_f8);
    (void)hipFree(d_tot);
    (void)hipFree(d_out);
    out[0] = best;
    out[1] = (double)tot;
    out[2] = rays[0];
    out[3] = rays[1];
    return RTG_OK;
#else
    g_err = "rtg_debug_replay: diagnostic builds only (RTG_DEBUG=1)";
    return RTG_ERR_ARG;
#endif
}

int rtg_synchronize(rtg_handle* h) {
    if (!h) return RTG_ERR_ARG;
    HIPOK(hipSetDevice(h->device));
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipStreamSynchronize(h->stream));
    float ms = 0;
    if (hipEventElapsedTime(&ms, h->ev[0], h->ev[1]) == hipSuccess) h->stats.render_ms = ms;
    return RTG_OK;
}

int rtg_film_read(rtg_handle* h, float* rgb, uint32_t* spp) {
    if (!h) return RTG_ERR_ARG;
    HIPOK(hipSetDevice(h->device));
    if (!rgb) {  // Film::SPP only: counts queued frames, waits for nothing
        if (spp) *spp = h->spp;
        return RTG_OK;
    }
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipStreamSynchronize(h->stream));
    if (rgb) HIPOK(hipMemcpy(rgb, h->d_film, (size_t)h->W * h->H * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (spp) *spp = h->spp;
    return RTG_OK;
}

int rtg_film_copy_device(rtg_handle* h, void* dst) {
    if (!h || !dst) return RTG_ERR_ARG;
    HIPOK(hipSetDevice(h->device));
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipMemcpyAsync(dst, h->d_film, (size_t)h->W * h->H * 3 * sizeof(float), hipMemcpyDeviceToDevice, h->stream));
    HIPOK(hipStreamSynchronize(h->stream));
    return RTG_OK;
}

int rtg_film_load(rtg_handle* h, const float* rgb, uint32_t spp) {
    if (!h || !rgb) return RTG_ERR_ARG;
    HIPOK(hipSetDevice(h->device));
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipStreamSynchronize(h->stream));  // (hipMemcpy does not order against non-blocking streams)
    HIPOK(hipMemcpy(h->d_film, rgb, (size_t)h->W * h->H * 3 * sizeof(float), hipMemcpyHostToDevice));
    h->spp = spp;
    return RTG_OK;
}

int rtg_clear(rtg_handle* h) {
    if (!h) return RTG_ERR_ARG;
    HIPOK(hipSetDevice(h->device));
    h->pend_n = 0;  // queued calls not issued yet: the clear would zero what they add
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipMemsetAsync(h->d_film, 0, (size_t)h->W * h->H * 3 * sizeof(float), h->stream));
    HIPOK(hipMemsetAsync(h->d_stats, 0, RTG_NSTATS * sizeof(unsigned long long), h->stream));
    HIPOK(hipStreamSynchronize(h->stream));
    h->spp = 0;
    h->stats = rtg_stats{};
    return RTG_OK;
}

int rtg_get_stats(rtg_handle* h, rtg_stats* out) {
    if (!h || !out) return RTG_ERR_ARG;
    HIPOK(hipSetDevice(h->device));
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipStreamSynchronize(h->stream));
    unsigned long long c[RTG_NSTATS] = {};
    HIPOK(hipMemcpy(c, h->d_stats, sizeof(c), hipMemcpyDeviceToHost));
    h->stats.node_visits = c[0];
    h->stats.tri_tests = c[1];
    h->stats.extension_rays = c[2];
    h->stats.shadow_rays = c[3];
    h->stats.shadow_node_visits = c[4];
    h->stats.shadow_tri_tests = c[5];
    h->stats.lane_slots = c[8];
    h->stats.node_lane_steps = c[9];
    h->stats.leaf_lane_steps = c[10];
    h->stats.leaf_phase_slots = c[13];
    h->stats.cullable_pops = c[11];
    h->stats.pops = c[12];
    h->stats.tri_tail_loads = c[6];
    h->stats.leafbox_tests = c[7];
    h->stats.traced_camera_rays = c[14];
    h->stats.lane_idle_no_ray = c[15];
    h->stats.lane_idle_last_leaf = c[16];
    h->stats.lane_idle_leaf_blocked = c[17];
    h->stats.lane_idle_retiring = c[18];
    h->stats.lane_idle_leaf_popped = c[19];
    *out = h->stats;
    return RTG_OK;
}

static int trace_query(rtg_handle* h, const float* rays, uint32_t n, float* hits, int32_t* vis, bool any) {
    if (!h || !rays || (!hits && !vis)) return RTG_ERR_ARG;
    if (n == 0) return RTG_OK;
    HIPOK(hipSetDevice(h->device));
    if (int rc = join_frames(h)) return rc;
    HIPOK(hipStreamSynchronize(h->stream));  // slot 0's overflow stack is free (hipMemcpy below)
    // path-id indirection of the trace kernels: identity queue over n query rays
    float4 *d_o = nullptr, *d_d = nullptr;
    unsigned* d_q = nullptr;
    void* d_out = nullptr;
    HIPOK(hipMalloc((void**)&d_o, (size_t)n * sizeof(float4)));
    HIPOK(hipMalloc((void**)&d_d, (size_t)n * sizeof(float4)));
    HIPOK(hipMalloc((void**)&d_q, (size_t)n * sizeof(unsigned)));
    HIPOK(hipMalloc(&d_out, (size_t)n * (any ? sizeof(int) : sizeof(float4))));
    {
        std::vector<float4> vo(n), vd(n);
        std::vector<unsigned> q(n);
        for (uint32_t i = 0; i < n; ++i) {
            const float* r = rays + (size_t)i * 8;
            vo[i] = make_float4(r[0], r[1], r[2], any ? r[3] : 0.0f);
            vd[i] = make_float4(r[4], r[5], r[6], 0.0f);
            q[i] = i;
        }
        HIPOK(hipMemcpy(d_o, vo.data(), (size_t)n * sizeof(float4), hipMemcpyHostToDevice));
        HIPOK(hipMemcpy(d_d, vd.data(), (size_t)n * sizeof(float4), hipMemcpyHostToDevice));
        HIPOK(hipMemcpy(d_q, q.data(), (size_t)n * sizeof(unsigned), hipMemcpyHostToDevice));
    }
    unsigned hc[4] = {n, 0, 0, 0};
    HIPOK(hipMemcpy(h->d_qctr, hc, sizeof(hc), hipMemcpyHostToDevice));
    int rc = ensure_ovf(h, h->slot[0]);
    if (rc) return rc;
    if (h->slot[0].stream) HIPOK(hipStreamSynchronize(h->slot[0].stream));
    TraceIO io{};
    io.fetch = h->d_qctr + 1;
    io.ovf = h->slot[0].d_ovf;
    io.stats = h->d_stats;
    io.cull = h->cull;
    io.wide = h->wide;
    if (any) {
        io.squeue = d_q;
        io.sray_o = d_o;
        io.sray_d = d_d;
        io.scount = h->d_qctr;
        io.visible = (int*)d_out;
    } else {
        io.queue = d_q;
        io.ray_o = d_o;
        io.ray_d = d_d;
        io.count = h->d_qctr;
        io.hits = (float4*)d_out;
    }
    if ((rc = launch_trace(h, io, h->stream))) return rc;
    HIPOK(hipStreamSynchronize(h->stream));
    if (any) HIPOK(hipMemcpy(vis, d_out, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
    else HIPOK(hipMemcpy(hits, d_out, (size_t)n * sizeof(float4), hipMemcpyDeviceToHost));
    (void)hipFree(d_o);
    (void)hipFree(d_d);
    (void)hipFree(d_q);
    (void)hipFree(d_out);
    return RTG_OK;
}

int rtg_probe_bsdf(const float* cases, uint32_t n, float* out) {
    if (!cases || !out) return RTG_ERR_ARG;
    if (n == 0) return RTG_OK;
    float *d_in = nullptr, *d_out = nullptr;
    HIPOK(hipMalloc((void**)&d_in, (size_t)n * 20 * sizeof(float)));
    HIPOK(hipMalloc((void**)&d_out, (size_t)n * 11 * sizeof(float)));
    HIPOK(hipMemcpy(d_in, cases, (size_t)n * 20 * sizeof(float), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_probe_bsdf, dim3((n + 255) / 256), dim3(256), 0, nullptr, d_in, (int)n, d_out);
    HIPOK(hipGetLastError());
    HIPOK(hipDeviceSynchronize());
    HIPOK(hipMemcpy(out, d_out, (size_t)n * 11 * sizeof(float), hipMemcpyDeviceToHost));
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return RTG_OK;
}

int rtg_probe_math(int fn, const float* in, uint32_t n, float* out) {
    if (!in || !out || fn < 0 || fn > 4 || n > 0x7fffffffu) return RTG_ERR_ARG;
    if (n == 0) return RTG_OK;
    const size_t nin = (size_t)n * (fn == 4 ? 2 : 1), nout = (size_t)n * (fn == 2 ? 2 : 1);
    float *d_in = nullptr, *d_out = nullptr;
    HIPOK(hipMalloc((void**)&d_in, nin * sizeof(float)));
    HIPOK(hipMalloc((void**)&d_out, nout * sizeof(float)));
    HIPOK(hipMemcpy(d_in, in, nin * sizeof(float), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_probe_math, dim3((n + 255) / 256), dim3(256), 0, nullptr, fn, d_in, (int)n, d_out);
    HIPOK(hipGetLastError());
    HIPOK(hipDeviceSynchronize());
    HIPOK(hipMemcpy(out, d_out, nout * sizeof(float), hipMemcpyDeviceToHost));
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return RTG_OK;
}

int rtg_trace_closest(rtg_handle* h, const float* rays, uint32_t n, float* hits) {
    return trace_query(h, rays, n, hits, nullptr, false);
}
int rtg_trace_visible(rtg_handle* h, const float* rays, uint32_t n, int32_t* visible) {
    return trace_query(h, rays, n, nullptr, visible, true);
}

}  // extern "C"
