// rtg_internal.h — declarations shared by the translation units of librtg.so (not part of the ABI):
// launch parameters of the wavefront kernels, the handle, and the host helpers that launch the
// traversal for the other integrators (rtg_kernels.hip: path tracer + traversal; rtg_light.hip:
// light tracing and instant radiosity, Renderer.h:82-326).
#pragma once
#include "rtg_dev.h"
#include "../../../include/rtg.h"

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

using namespace rtgd;

#define RTG_TB 256          // threads per block (4 waves)
#define RTG_POP ((int)0x80000001)  // "pop the stack" marker inside one traversal step
#ifndef RTG_STACK
#define RTG_STACK 24        // per-lane traversal stack entries kept in LDS (24 KB per block)
#endif
#ifndef RTG_POSTPONE
#define RTG_POSTPONE 32     // >0: park a reached leaf and keep walking; run the leaves of a wave together
#endif                      //     once this many lanes hold one (or no lane can walk on)
#ifndef RTG_DRAIN_LEAF
#define RTG_DRAIN_LEAF 1    // once the queue is empty, run the leaf phase whenever a lane has parked a
#endif                      //     leaf (the drain is latency-bound: lanes should not wait for each other)
#ifndef RTG_REFILL
#define RTG_REFILL 12       // refill idle lanes once at least this many are idle (the setup code then
#endif                      // runs with more lanes per execution)
#ifndef RTG_SLICE_MIX
#define RTG_SLICE_MIX 1     // 1: each of the 8 work slices = an eighth of the extension rays, then an
#endif                      //    eighth of the shadow rays (k_trace)
#ifndef RTG_TRI_SPLIT
#define RTG_TRI_SPLIT 1     // triangle record: two dwordx4 for t, the third only for a candidate t
#endif
#ifndef RTG_TRACE_WPE
#define RTG_TRACE_WPE 6     // minimum waves per SIMD requested for the traversal kernel
#endif
#define RTG_CULL_REL 1.52587890625e-05f  // 2^-16 relative inflation for distance culling
#ifndef RTG_FETCH
#define RTG_FETCH 256       // rays a wave takes from the work counter per atomic (k_trace pool; 64: -3.5 %)
#endif
#ifndef RTG_FETCH_TAIL
#define RTG_FETCH_TAIL 8    // k: fetch 64 rays per atomic once about k rounds of big batches are left
#endif
#ifndef RTG_TAIL_BATCH
#define RTG_TAIL_BATCH 64   // rays per atomic in the tail rounds
#endif
#ifndef RTG_WAVETIME
#define RTG_WAVETIME 0      // 1: compile k_trace's per-wave clocks (diagnostic; RTG_WAVETIME env then enables)
#endif
#ifndef RTG_COLLAPSE_DP
#define RTG_COLLAPSE_DP 0   // 1: SAH-optimal BVH2 -> 4-wide cut with leaf merging (env RTG_COLLAPSE=dp|greedy)
#endif
#ifndef RTG_GEN_LEAN
#define RTG_GEN_LEAN 1      // bounce-0 path state implied instead of written by k_generate (ChunkArgs::lean)
#endif
#ifndef RTG_SHC_SPEC
#define RTG_SHC_SPEC 1      // k_shade stores the NEE value in contrib up front; k_trace clears it on occlusion
#endif
#ifndef RTG_SHADE_PF
#define RTG_SHADE_PF 0      // 1: k_shade loads the next iteration's path id one iteration ahead
#endif
#ifndef RTG_REBUILD
#define RTG_REBUILD 1       // wide nodes cut from an own 3-axis SAH tree over the reference leaves (env RTG_REBUILD=0: from the reference BVH2)
#endif
#ifndef RTG_FETCH8
#define RTG_FETCH8 1        // k_trace fetches from 8 slice counters (TraceIO::fetch8): +4 % per GPU at N=8
#endif
#ifndef RTG_FETCH_ADAPT
#define RTG_FETCH_ADAPT 0   // 1: big batch = min(RTG_FETCH, ~1/16 of a wave's share) (no gain)
#endif
#ifndef RTG_SHADE_BUF
#define RTG_SHADE_BUF 0     // >0: k_shade stages compacted path ids in LDS (entries per queue) and
                            // appends them with one atomic per flush instead of one per 256 paths
#endif
#ifndef RTG_FAST_PUSH
#define RTG_FAST_PUSH 1     // wide-node pushes as three unconditional LDS writes when they fit (~1 %)
#endif
#ifndef RTG_SEL_SORT
#define RTG_SEL_SORT 0      // 1: slot sort network as selects instead of branches
#endif
#ifndef RTG_SHADE_SORT
#define RTG_SHADE_SORT 0    // 1: k_shade partitions each block's paths into misses and hits first (C3: no change)
#endif
#ifndef RTG_SHADE_WAVES
#define RTG_SHADE_WAVES 5                // min waves per SIMD for k_shade (96 VGPRs, no spills)
#endif

// Work counters of one bounce. Every field sits in its own 128-B line (RTG_CTR_PAD): the
// device-scope atomics on them (queue appends in k_shade, work fetches in k_trace) are served one
// line at a time, so counters sharing a line serialise with each other.
#ifndef RTG_CTR_PAD
#define RTG_CTR_PAD 1
#endif
#if RTG_CTR_PAD
#define RTG_CPAD(f) unsigned f; unsigned f##_pad[31];
#else
#define RTG_CPAD(f) unsigned f;
#endif
struct __align__(16) Counters {
    RTG_CPAD(n_ext) RTG_CPAD(n_shadow) RTG_CPAD(f_ext) RTG_CPAD(f_shadow) RTG_CPAD(f_shade) RTG_CPAD(pad0)
    RTG_CPAD(pad1) RTG_CPAD(pad2)
    unsigned f8[8 * 32];  // sliced work counters of k_trace (TraceIO::fetch8), one 128-B line each
};
#undef RTG_CPAD

// Queues hold path ids only; ray payloads live in per-path arrays (written in place by k_shade),
// so compaction moves 4 bytes per ray and needs one atomic per 256 paths.
// One traversal launch serves two ray sets: extension (closest-hit) rays take work indices
// [0, nc) and NEE shadow (any-hit) rays [nc, nc + ns). Each lane carries its ray's kind.
struct TraceIO {
    const unsigned* queue;     // closest: path ids to trace
    const float4* ray_o;       // closest: [pid] origin.xyz
    const float4* ray_d;       // closest: [pid] direction.xyz
    const unsigned* count;     // closest: number of rays (device; null = none)
    float4* hits;              // closest-hit output [pid]
    const unsigned* squeue;    // any-hit: path ids
    const float4* sray_o;      // any-hit: [pid] origin.xyz, w = maxT
    const float4* sray_d;      // any-hit: [pid] direction.xyz
    const float4* sray_c;      // any-hit: [pid] NEE value copied to contrib[pid] when visible
    const unsigned* scount;    // any-hit: number of rays (device; null = none)
    float4* contrib;           // any-hit: this bounce's contribution plane [pid]
    int* visible;              // any-hit query output [pid] (instead of contrib)
    unsigned* fetch;           // work counter over both sets (device, zeroed)
    unsigned* fetch8;          // or (non-null) 8 slice counters at a stride of 32 (device, zeroed)
    int* ovf;                  // global stack overflow [level][thread]
    unsigned long long* stats; // [0,1] closest / [4,5] any-hit: box tests, triangle tests (COUNT)
    int cull;
    int wide;                  // traverse the 4-wide tree when the ray allows it
    unsigned long long* wtime; // diagnostics (RTG_WAVETIME): per wave start / drained / exit clock
    float4 cam_o;              // closest: the origin of every ray when ray_o is null (camera rays);
                               // a null queue is the identity (path id = ray index)
};

struct ChunkArgs {
    const unsigned* pixlist;   // local pixel -> pixel index (y*W + x)
    unsigned npix, ns, s0, P;
    unsigned long long seed;
    int max_depth;
    int mode;                  // RTG_INTEGRATOR_* (first-hit estimators never continue a path)
    int pm;                    // path id order: 1 pixel-major (pid = lp * ns + sl), 0 sample-major
    DevCamera cam;
    int lean = 0;              // 1: bounce-0 state implied (identity queue, camera origin, thr 1,
                               // PCG seed, canHitLight); k_generate writes ray_d only
};

struct PathBufs {
    float4* thr;               // [P] throughput
    unsigned long long* rng;   // [P] PCG state
    int* meta;                 // [P] nterms | canHitLight << 8
    float4* contrib;           // [maxb][P] per-vertex radiance terms
    float4* ray_o;             // [P] current extension ray origin
    float4* ray_d;             // [P] current extension ray direction
    float4* hits;              // [P] its closest hit (t, id, alpha, beta)
    float4* sh_o;              // [P] NEE shadow ray origin + maxT
    float4* sh_d;              // [P] NEE shadow ray direction
    float4* sh_c;              // [P] NEE value thr * Ld if visible
    unsigned* q[2];            // extension queues of path ids (ping-pong)
    unsigned* shq;             // shadow queue of path ids
    Counters* ctr;             // [maxb + 1]
};

static __device__ __forceinline__ int lane_id() { return __lane_id(); }
static __device__ __forceinline__ unsigned prefix_lt(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}



// ------------------------------------------------------------------ host side
extern thread_local std::string g_err;

#define HIPOK(expr)                                                                          \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            g_err = std::string(#expr) + ": " + hipGetErrorString(e_);                       \
            return RTG_ERR_HIP;                                                              \
        }                                                                                    \
    } while (0)
#define LAUNCH_OK(name)                                                                      \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ != hipSuccess) {                                                              \
            g_err = std::string("launch ") + name + ": " + hipGetErrorString(e_);            \
            return RTG_ERR_HIP;                                                              \
        }                                                                                    \
    } while (0)



template <class T>
static int dev_upload(T** dst, const std::vector<T>& src) {
    *dst = nullptr;
    size_t bytes = std::max<size_t>(src.size(), 1) * sizeof(T);
    HIPOK(hipMalloc((void**)dst, bytes));
    if (!src.empty()) HIPOK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return RTG_OK;
}

struct rtg_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    int W = 0, H = 0;
    uint32_t spp = 0;
    int max_depth = 4, cull = 1, count = 0, timing = 0;
    uint32_t max_paths = 1u << 30;  // 1G paths in flight at most; the chunk is held to half the free HBM
    int n_cu = 256, trace_blocks = 0, trace_blocks_count = 0, shade_blocks = 0, packet_blocks = 0;
    int fetch8 = RTG_FETCH8;  // sliced work counters for k_trace (RTG_FETCH8 env overrides)
    int pixel_major = 1;  // path ids pixel-major: a wave's rays share pixels (RTG_PIXEL_MAJOR=0: sample-major)
    int packet = 0;  // RTG_PACKET=1: camera rays by the packet walk (exact, but slower: DESIGN.md §4)
    uint32_t bvh_depth = 0;
    SceneView sv{};
    DevCamera cam{};
    rtg_camera_proj proj{};  // projectOntoCamera state (light tracing, rtg_light.hip)
    DevNode* d_nodes = nullptr;
    DevNodeW* d_nodesw = nullptr;
    DevNodeQ* d_nodesq = nullptr;
    float4* d_leafbox = nullptr;
    int usew = 0, wide = 1;
    int integrator = RTG_INTEGRATOR_PATH;
    bool rebuilt = false;     // wide tree cut from rebuild_over_leaves (RTG_REBUILD)
    uint32_t wide_depth = 0;  // wide levels on the longest root-to-leaf path
    DevTri* d_tris = nullptr;
    DevTri48* d_tris48 = nullptr;
    DevShade* d_shade = nullptr;
    DevMat* d_mats = nullptr;
    DevLight* d_lights = nullptr;
    DevTex* d_texinfo = nullptr;
    float* d_texels = nullptr;
    float* d_film = nullptr;
    // chunk buffers
    // two chunk pipelines (buffers, stream, overflow region each): pipeline 1 runs on stream2
    size_t cap_P[2] = {0, 0};
    int cap_maxb[2] = {0, 0};
    PathBufs pb[2]{};
    hipStream_t stream2 = nullptr;
    int pipes = 1, stagger = 2;
    int shade_grid = 1;  // RTG_SHADE_GRID: k > 0: P / (256 k) blocks of k tiles each; 0: persistent (n_cu x occupancy)
    hipEvent_t pev[4] = {nullptr, nullptr, nullptr, nullptr};  // fork, stagger, join, accumulate-order
    unsigned* d_pix = nullptr;
    size_t cap_pix = 0;
    std::vector<uint32_t> pix_key;
    unsigned npix = 0;
    int* d_ovf = nullptr;
    size_t cap_ovf = 0;
    unsigned* d_qctr = nullptr;  // query-API counters [4]
    unsigned long long* d_stats = nullptr;
    rtg_stats stats{};
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> kev;  // per-launch timing events (timing mode)
};


// rtg_kernels.hip
int ensure_ovf(rtg_handle* h);
int set_pixels(rtg_handle* h, const uint32_t* tiles, uint32_t n_tiles);
int ensure_chunk(rtg_handle* h, int i, size_t P, int maxb);
int render_impl(rtg_handle* h, uint32_t first, uint32_t n_samples, uint64_t seed, const uint32_t* tiles,
                uint32_t n_tiles, hipStream_t st);
// k_generate for the paths of a (camera rays at pixel centres, Scene.h:43-54)
int launch_generate(rtg_handle* h, const ChunkArgs& a, const PathBufs& pb, hipStream_t st);
// one k_trace launch (closest-hit rays of io.queue and any-hit rays of io.squeue) on stream st
int launch_trace(rtg_handle* h, const TraceIO& io, hipStream_t st);
