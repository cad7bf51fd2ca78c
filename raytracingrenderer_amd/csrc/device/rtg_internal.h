// rtg_internal.h — declarations shared by the translation units of librtg.so (not part of the ABI):
// launch parameters of the wavefront kernels, the handle, and the host helpers that launch the
// traversal for the other integrators (rtg_kernels.hip: path tracer + traversal; rtg_light.hip:
// light tracing and instant radiosity, Renderer.h:82-326).
#pragma once
#include "rtg_dev.h"
#include "../../../include/rtg.h"

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <string>
#include <vector>

using namespace rtgd;

#define RTG_TB 256          // threads per block (4 waves)
#define RTG_NSTATS 24       // device counters behind rtg_stats (rtg_handle::d_stats)
#ifndef RTG_TTB
#define RTG_TTB 64          // threads per k_trace block: one wave, so a drained wave gives its CU slot
                            // back at once (256: C3 -0.4 %, shard-of 8 -0.6 %, profiles/r03_trace_block_ab.txt)
#endif
#define RTG_POP ((int)0x80000001)  // "pop the stack" marker inside one traversal step
// Measured constants of the traversal and shading kernels (DESIGN.md §4 records the A/B runs;
// the rejected alternatives are archived under tools/experiments/, not compiled in):
#ifndef RTG_STACK
#define RTG_STACK 16        // per-lane traversal stack entries kept in LDS (64 B per lane; deeper entries
#endif                      // go to the global overflow). 16 keeps a one-wave block at 4.1 KB of LDS for
                            // 7 blocks per SIMD (20 entries: slower, 24: 6 per SIMD)
// (the tuning constants are overridable with -D for A/B builds: tools/ab_matrix.sh)
#ifndef RTG_STACK_SMALL
#define RTG_STACK_SMALL 7   // the LDS stack of k_trace's small-scene variant (with its scene image in LDS)
#endif
#ifndef RTG_SMALL_F4
#define RTG_SMALL_F4 192    // small-scene image limit, float4s (3 KB; cornell's SBVH image is 188): with
#endif                      // 7 x 256 B of stack a one-wave block takes 4.9 KB, 28 blocks (7 waves) per CU
                            // (224 float4s and 11 entries: 6.5 KB, 6 waves; C2 walk -7 %)
#ifndef RTG_SMALL_LB
#define RTG_SMALL_LB 0      // 1: the small-scene image holds the leaf boxes too; 0: they stay in global
#endif                      // memory, read once per candidate hit (C2 +4.8 %: cornell's SBVH image then fits)
#ifndef RTG_CAM_GRID
#define RTG_CAM_GRID 1      // the camera launch runs at most one one-wave block per 64 rays (its one
#endif                      // work counter then takes no probes from waves without work; +0.5 %)
#ifndef RTG_POSTPONE
#define RTG_POSTPONE 32     // park a reached leaf and keep walking; run the leaves of a wave together
                            // once this many lanes hold one (or no lane can walk on, or the queue is dry)
#endif
#ifndef RTG_MEM_PCT
#define RTG_MEM_PCT 50      // percent of the free HBM the path state of the chunks in flight may take (60:
                            // C5's 32-spp step in one chunk, +3 % once allocated, but allocations past
                            // ~half the VRAM take seconds: a one-shot C5 frame 4.8 -> 8.4 s)
#endif
#ifndef RTG_PEND2
#define RTG_PEND2 1         // a lane parks a second reached leaf instead of idling until the leaf phase
#endif                      // (node-step lane use 0.70 -> 0.77 on C3: +1 to +2 %)
#ifndef RTG_REFILL
#define RTG_REFILL 12       // refill idle lanes once at least this many are idle (the setup code then
                            // runs with more lanes per execution)
#endif
#ifndef RTG_TRACE_WPE
#define RTG_TRACE_WPE 7     // minimum waves per SIMD requested for the traversal kernel: <= 72 VGPRs and
#endif                      // <= 96 SGPRs (its unit is built without SLP vectorisation: 64 VGPRs, no spills)
#define RTG_CULL_REL 1.52587890625e-05f  // 2^-16 relative inflation for distance culling
#ifndef RTG_FETCH
#define RTG_FETCH 256       // rays a wave takes from a work counter per atomic (k_trace pool)
#endif
#ifndef RTG_FETCH_TAIL
#define RTG_FETCH_TAIL 8    // fetch RTG_TAIL_BATCH rays per atomic once about this many rounds of
#endif                      // big batches are left in the slice (shorter drain tails)
#ifndef RTG_TAIL_BATCH
#define RTG_TAIL_BATCH 64
#endif
#ifndef RTG_LDS_MATS
#define RTG_LDS_MATS 64     // k_shade holds the material table in LDS up to this many records (64 B each)
#endif
#ifndef RTG_LDS_LIGHTS
#define RTG_LDS_LIGHTS 48   // ... and the light table up to this many (80 B each): 5 x 48 < 256 threads
#endif
#ifndef RTG_SHADE_WAVES
#define RTG_SHADE_WAVES 7   // min waves per SIMD for k_shade (72 VGPRs, no spills; one tile per block)
#endif
// The own binary tree the wide nodes are cut from (prepare_scene; rtg_bvh.hip for spatial splits)
#ifndef RTG_SAH_SWEEP
#define RTG_SAH_SWEEP 2048  // full SAH sweep up to this many primitives in a node, binned above
#endif
#ifndef RTG_SAH_BINS
#define RTG_SAH_BINS 128    // centroid bins per axis of the binned SAH (64: C5 -2.3 %)
#endif
#ifndef RTG_SBVH
#define RTG_SBVH 1          // spatial splits (rtg_bvh.hip build_sbvh); 0: object splits only
#endif
#ifndef RTG_UNIFORM_TEX
#define RTG_UNIFORM_TEX 1   // constant textures of any size take the 1x1 path (no texel fetches)
#endif
#ifndef RTG_SBVH_BINS
#define RTG_SBVH_BINS 32    // slabs per axis of a spatial split
#endif
#ifndef RTG_SBVH_ALPHA
#define RTG_SBVH_ALPHA 1e-5 // spatial splits are tried when the object split's two boxes overlap by
#endif                      // more than this fraction of the root box's area
#ifndef RTG_SBVH_DUP
#define RTG_SBVH_DUP 0.5    // at most this many extra references per triangle in all
#endif
// RTG_DEBUG=1 (a diagnostic build only) compiles k_trace's per-wave clocks (RTG_OPT_WAVETIME) and
// the fetch capture + replay of the locality-matched roofline (RTG_OPT_CAPTURE, rtg_debug_replay).
#define RTG_CAP_LEN 64
#ifndef RTG_DEBUG
#define RTG_DEBUG 0
#endif

// Work counters of one bounce. Every field sits in its own 128-B line: the device-scope atomics on
// them (queue appends in k_shade, work fetches in k_trace) are served one line at a time, so
// counters sharing a line serialise with each other.
#define RTG_CPAD(f) unsigned f; unsigned f##_pad[31];
struct __align__(16) Counters {
    RTG_CPAD(n_ext) RTG_CPAD(n_shadow) RTG_CPAD(f_ext) RTG_CPAD(f_shadow) RTG_CPAD(f_shade)
    RTG_CPAD(n_cam)  // path tracer, bounce 0: camera rays traced, one per pixel (k_generate)
    RTG_CPAD(pad1) RTG_CPAD(pad2)
    unsigned f8[8 * 32];  // sliced work counters of k_trace (TraceIO::fetch8), one 128-B line each
    // path tracer queues, segmented: k_shade block t appends to segment t % 8 (a device-scope atomic
    // on one counter serialises at ~87M/s: one counter for all blocks made k_shade atomic-bound,
    // tools/micro/atomic.hip); segment k holds ne8[32k] extension / ns8[32k] shadow rays from
    // queue position k * seg_cap (ChunkArgs::seg_cap), and is k_trace's slice k
    unsigned ne8[8 * 32];
    unsigned ns8[8 * 32];
};
#undef RTG_CPAD
// positions of a segmented queue for P paths: 8 segments of ceil(ceil(P / 256) / 8) tiles of 256
static inline size_t seg_tiles(size_t P) { return ((P + 255) / 256 + 7) / 8; }
static inline size_t queue_slots(size_t P) { return seg_tiles(P) * 8 * 256; }

// A ray's payload sits at its queue position (PathBufs); compaction needs one atomic per 256 paths.
// One traversal launch serves two ray sets: extension (closest-hit) rays take work indices
// [0, nc) and NEE shadow (any-hit) rays [nc, nc + ns). Each lane carries its ray's kind.
struct TraceIO {
    const unsigned* queue;     // closest: path ids to trace (null: the ray at position i is path i;
                               // the path tracer keeps its extension payload in queue order)
    const float4* ray_o;       // closest: [pid] origin.xyz
    const float4* ray_d;       // closest: [pid] direction.xyz
    const unsigned* count;     // closest: number of rays (device; null = none)
    float4* hits;              // closest-hit output [pid]
    const unsigned* squeue;    // any-hit: path ids
    const float4* sray_o;      // any-hit: [pid] origin.xyz, w = maxT
    const float4* sray_d;      // any-hit: [pid] direction.xyz
    const float4* sray_c;      // any-hit: [pid] NEE value copied to contrib[pid] when visible
    int spos;                  // any-hit rays (sray_o, sray_d) at their shadow-queue position (path
                               // tracer); 0: by path id (light tracer, queries)
    const unsigned* scount;    // any-hit: number of rays (device; null = none)
    float4* contrib;           // any-hit: this bounce's contribution plane [pid]
    int* visible;              // any-hit query output [pid] (instead of contrib)
    unsigned* fetch;           // work counter over both sets (device, zeroed)
    unsigned* fetch8;          // or (non-null) 8 slice counters at a stride of 32 (device, zeroed)
    unsigned seg_cap;          // != 0: segmented queues (path tracer, bounce >= 1): slice k = the
                               // seg_ne[32k] extension rays at positions k * seg_cap.. then the
                               // seg_ns[32k] shadow rays at shadow positions k * seg_cap..; the
                               // extension index span `count` is then 8 * seg_cap
    const unsigned* seg_ne;    // (null: no extension rays)
    const unsigned* seg_ns;    // (null: no shadow rays)
    int* ovf;                  // global stack overflow [level][thread]
    unsigned long long* stats; // [0,1] closest / [4,5] any-hit: box tests, triangle tests (COUNT)
    int cull;
    int wide;                  // traverse the 4-wide tree when the ray allows it
    unsigned long long* wtime; // RTG_DEBUG builds: per wave start / drained / exit clock
    uint4* cap;                // RTG_DEBUG builds (RTG_OPT_CAPTURE): every ray's record fetches,
                               // [k / 4][ray] uint4 (type << 30 | index; type 0 wide node, 1 triangle
                               // head, 2 leaf box, 3 BVH2 node), at most RTG_CAP_LEN per ray
    unsigned* cap_len;         // [ray] fetches captured (<= RTG_CAP_LEN)
    unsigned cap_n;            // rays the capture holds (work index space of the launch)
    float4 cam_o;              // closest: the origin of every ray when ray_o is null (camera rays);
                               // a null queue is the identity (path id = ray index)
    unsigned* hcnt;            // non-null (big waited-for chunks): block 0 stores the 8 extension
                               // segment counts (seg_ne) here as the launch starts, with system-scope
                               // stores to host-coherent memory, and the host sizes the next k_shade
                               // grid from them (rtg_handle::h_cnt) without a device-to-host copy
};

struct ChunkArgs {
    const unsigned* pixlist;   // local pixel -> pixel index (y*W + x)
    unsigned npix, ns, s0, P;
    unsigned long long seed;
    int max_depth;
    int mode;                  // RTG_INTEGRATOR_* (first-hit estimators never continue a path)
    DevCamera cam;
    int lean = 0;              // 1: bounce-0 state implied (identity queue, camera origin, thr 1,
                               // PCG seed, canHitLight); k_generate writes ray_d only
    unsigned seg_tiles = 0;    // tiles of 256 per queue segment (Counters::ne8); k_shade grid = 8x
    // path ids are pixel-major: pid = lp * ns + sl (a wave of camera rays is one pixel's samples)
    unsigned long long ns_mul = 0;  // lp = (pid * ns_mul) >> ns_shift (set_ns_div); 0: divide
    unsigned ns_shift = 0;
};
// pid / ns as a multiply. With 2^l >= ns, S = 31 + l and M = ceil(2^S / ns) < 2^32, the excess
// e = M ns - 2^S < ns <= 2^l. Writing pid = q ns + r, pid M / 2^S = q + r / ns + pid e / (ns 2^S),
// and the last two terms stay below 1 when pid e < 2^S, i.e. for every pid < 2^31: the floor is q.
static inline void set_ns_div(ChunkArgs& a) {
    a.ns_mul = 0;
    if ((unsigned long long)a.P > (1ull << 31)) return;
    unsigned l = 0;
    while ((1u << l) < a.ns) ++l;
    const unsigned S = 31 + l;
    a.ns_mul = ((1ull << S) + a.ns - 1) / a.ns;
    a.ns_shift = S;
}
static __device__ __forceinline__ void split_pid(const ChunkArgs& a, unsigned pid, unsigned& lp, unsigned& sl) {
    lp = a.ns_mul ? (unsigned)(((unsigned long long)pid * a.ns_mul) >> a.ns_shift) : pid / a.ns;
    sl = pid - lp * a.ns;
}

struct PathBufs {
    // extension payload, two sets (the path tracer's bounce b reads set b & 1 by queue position and
    // writes set (b + 1) & 1; the light tracer / instant radiosity use set 0 by path id)
    float4* thr;               // [P] throughput (.w: computeDirectMIS's BSDF pdf)
    unsigned long long* rng;   // [P] PCG state
    float4* ray_o;             // [P] extension ray origin (.w: path id, path tracer)
    float4* ray_d;             // [P] extension ray direction (.w: canHitLight, path tracer)
    float4* thr2;              // set 1
    unsigned long long* rng2;
    float4* ray_o2;
    float4* ray_d2;
    int* meta;                 // [P] by path id: nterms | canHitLight << 8
    float4* contrib;           // [maxb][P] by path id: per-vertex radiance terms
    float4* hits;              // [P] closest hit (t, id, alpha, beta) of the ray at queue position i
    float4* sh_o;              // [P] NEE shadow ray origin + maxT (path tracer: at its shadow-queue position)
    float4* sh_d;              // [P] NEE shadow ray direction (same)
    float4* sh_c;              // [P] by path id: NEE value thr * Ld if visible
    unsigned* q[2];            // extension queues of path ids (ping-pong; light tracer and instant
                               // radiosity only, allocated on their request: ensure_chunk(queues))
    unsigned* shq;             // shadow queue of path ids
    Counters* ctr;             // [maxb + 1]
};

static __device__ __forceinline__ int lane_id() { return __lane_id(); }
static __device__ __forceinline__ unsigned prefix_lt(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}



// ------------------------------------------------------------------ host side
extern thread_local std::string g_err;

// roctx ranges around the host-side stages of a render (generate / trace(b) /
// shade(b) / accumulate); rocprofv3 --marker-trace shows them beside the kernel trace. A range
// spans the enqueue of its launches (the kernels themselves are in the kernel trace).
struct RoctxRange {
    explicit RoctxRange(const char* m) { roctxRangePushA(m); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};
// "rtg:trace b=<b>" / "rtg:shade b=<b>" names for b < 32 (static strings: roctx copies nothing)
const char* roctx_stage_name(int kind, int b);

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

// Chunks in flight (the frame pipeline). A chunk of at most RTG_PIPE_MAX_P paths -- e.g. queued 1-spp
// frames of the drop-in RayTracer::render() flushed before RTG_COALESCE_P -- is issued without any host wait (its
// k_shade grids cover every tile a segment can hold; blocks past the live count exit at once) into the
// next of RTG_SLOTS slots, each with its own path state, stack overflow and stream, so consecutive
// frames run side by side on the GPU and fill each other's drain tails. The film folds stay in sample
// order: a chunk's k_accumulate waits for the previous chunk's (rtg_handle::last_fold). Larger chunks
// run in slot 0 alone and size each k_shade grid from the live counts read back during the
// traversal (a grid of every possible tile costs more than the wait there).
#ifndef RTG_SLOTS
#define RTG_SLOTS 3                        // with the handle's stream, 4 = GPU_MAX_HW_QUEUES streams
#endif
#ifndef RTG_PIPE_MAX_P
#define RTG_PIPE_MAX_P (16u << 20)
#endif
#ifndef RTG_COALESCE_P
#define RTG_COALESCE_P (64u << 20)         // queued frames are issued once this many paths are pending
                                           // (64 frames of 1 Mpixel: one chunk, like the batched render)
#endif
#ifndef RTG_HOSTGRID_MIN_TILES
#define RTG_HOSTGRID_MIN_TILES 4096u       // big chunks: seg_tiles at or above this size the k_shade grid
#endif                                     // from the read-back counts
struct ChunkSlot {
    PathBufs pb{};
    size_t cap_P = 0;           // paths the buffers hold
    int cap_maxb = 0;           // contribution planes they hold
    int* d_ovf = nullptr;       // k_trace's stack overflow [level][thread] for launches of this slot
    size_t cap_ovf = 0;
    hipStream_t stream = nullptr;
    hipEvent_t fold = nullptr;  // this slot's last film fold (k_accumulate) has run
    bool used = false;          // fold has been recorded
};

struct rtg_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    int W = 0, H = 0;
    uint32_t spp = 0;
    int max_depth = 4, cull = 1, count = 0, timing = 0, serial = 0;
    uint32_t max_paths = 1u << 30;  // 1G paths in flight at most; the chunk is held to half the free HBM
    size_t mem_cap = 0;  // != 0: path-state budget of this handle (a group rehearsing k ranks on one
                         // device gives each 1/k of half the device's free HBM, so their chunks match)
    int n_cu = 256, trace_blocks = 0, trace_blocks_count = 0, trace_blocks_small = 0, trace_blocks_small_count = 0;
    int wavetime = 0;  // RTG_DEBUG builds: per-wave clocks of the first chunk (RTG_OPT_WAVETIME)
    int capture_launch = -1;  // RTG_DEBUG builds: trace launch of chunk 0 whose fetches are captured
    uint4* d_cap = nullptr;           // its chains (TraceIO::cap)
    unsigned* d_cap_len = nullptr;    // its chain lengths
    unsigned* d_cap_rays = nullptr;   // [2]: its extension and shadow ray counts
    unsigned cap_n = 0;               // rays the capture buffers hold
    std::vector<double> launch_ms;    // per trace launch of the last timed render (RTG_OPT_TIMING)
    std::vector<unsigned long long> launch_rays;  // rays of each trace launch of its last chunk
    uint32_t bvh_depth = 0;
    SceneView sv{};
    DevCamera cam{};
    rtg_camera_proj proj{};  // projectOntoCamera state (light tracing, rtg_light.hip)
    DevNode* d_nodes = nullptr;
    DevNodeQ* d_nodesq = nullptr;
    float4* d_leafbox = nullptr;
    float4* d_img = nullptr;   // the small-scene image (SceneView::img)
    int usew = 0, wide = 1;
    int integrator = RTG_INTEGRATOR_PATH;
    bool rebuilt = false;     // wide tree cut from rebuild_over_leaves (else from the reference BVH2)
    uint32_t wide_depth = 0;  // wide levels on the longest root-to-leaf path
    DevTri48* d_tris48 = nullptr;
    DevShade* d_shade = nullptr;
    DevMat* d_mats = nullptr;
    DevLight* d_lights = nullptr;
    DevTex* d_texinfo = nullptr;
    float* d_texels = nullptr;
    float* d_film = nullptr;
    // chunk buffers (path state of the paths in flight), one set per slot; slot 0 also serves the
    // light tracer, instant radiosity and the ray queries (on `stream`)
    ChunkSlot slot[RTG_SLOTS];
    unsigned next_slot = 0;        // the pipeline's next slot
    hipEvent_t entry = nullptr;    // recorded on the caller's stream when a render starts: chunks wait on it
    hipEvent_t last_fold = nullptr;  // the last queued chunk's fold (a slot's event; null before any)
    bool inflight = false;         // chunks queued by rtg_render_async(.., NULL) not yet joined to `stream`
    // queued calls not yet issued (rtg_render_async with no stream): consecutive calls of the same
    // seed and tiles whose samples follow on are coalesced into one chunk of up to RTG_COALESCE_P
    // paths, issued when that fills or when anything reads, waits or changes a setting
    uint32_t pend_first = 0, pend_n = 0;
    uint64_t pend_seed = 0;
    std::vector<uint32_t> pend_key;
    int no_coalesce = 0;           // RTG_OPT_NO_COALESCE: every queued call is issued at once
    unsigned* d_pix = nullptr;
    size_t cap_pix = 0;
    std::vector<uint32_t> pix_key;
    unsigned npix = 0;
    unsigned* d_qctr = nullptr;  // query-API counters [4]
    unsigned long long* d_stats = nullptr;
    rtg_stats stats{};
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> kev;  // per-launch timing events (timing mode)
    // k_shade's grid (big waited-for chunks): the 8 segment counts of bounce b's extension queue,
    // stored into host-coherent memory by k_trace(b)'s block 0 as it starts (TraceIO::hcnt; 8 per
    // bounce, RTG_CNT_PENDING until written), so the host launches k_shade(b) while k_trace(b) runs.
    // (Until round 5 a hipMemcpyAsync on a side stream read them back: its blit kernel queued behind
    // the persistent k_trace for a CU slot, ~4.7 ms per copy, and the host launch waited for it.)
    unsigned* h_cnt = nullptr;
    unsigned* d_hcnt = nullptr;   // the same memory, device address
    int cap_cnt = 0;
    std::vector<hipEvent_t> tev;  // [b]: k_trace(b) has finished (a launch that never wrote its counts)
};
#define RTG_CNT_PENDING 0xFFFFFFFFu


// The device records of a scene, built on the host from an rtg_scene_desc (prepare_scene) and
// uploaded per device (upload_scene); rtg_create does both, a group prepares once.
struct HostScene {
    std::vector<DevNode> nodes;
    std::vector<DevNodeQ> nodesq;
    std::vector<float4> leafbox;
    std::vector<float4> img;   // small scenes: [wide nodes | triangles | leaf boxes] (SceneView::img)
    int img_tri = 0, img_lb = 0;
    std::vector<DevTri48> tris48;
    std::vector<DevShade> shade;
    std::vector<DevMat> mats;
    std::vector<DevLight> lights;
    std::vector<DevTex> texinfo;
    std::vector<float> texels;
    int n_lights = 0, env_tex = -1, env_off = 0, env_w = 1, env_h = 1;
    bool env_uniform = false;  // every texel of the environment map has the same bits
    float env_one[3] = {0.0f, 0.0f, 0.0f};
    int root_word = RTG_EXIT, root_wordw = RTG_EXIT;
    bool usew = false, rebuilt = false;
    uint32_t bvh_depth = 0, wide_depth = 0;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    float cull_scale = 0.0f;
    DevCamera cam{};
    rtg_camera_proj proj{};
};

// rtg_bvh.hip: the own binary tree with spatial splits over the triangles (descriptor node format)
bool build_sbvh(const rtg_scene_desc* d, std::vector<int32_t>& lk, std::vector<float>& bd);
// rtg_kernels.hip
int prepare_scene(const rtg_scene_desc* d, HostScene& hs);
int upload_scene(int device, const HostScene& hs, rtg_handle* h);
int ensure_ovf(rtg_handle* h, ChunkSlot& sl);
int set_pixels(rtg_handle* h, const uint32_t* tiles, uint32_t n_tiles);
// path state of P paths with maxb contribution planes in slot sl (+ the id queues q[0..1] if asked)
int ensure_chunk(rtg_handle* h, ChunkSlot& sl, size_t P, int maxb, bool queues);
// lazy: chunks stay queued past the return (rtg_render_async with no stream); join_frames later makes
// the handle's stream wait for them. Otherwise `st` waits for them before render_impl returns.
int render_impl(rtg_handle* h, uint32_t first, uint32_t n_samples, uint64_t seed, const uint32_t* tiles,
                uint32_t n_tiles, hipStream_t st, bool lazy, bool add_spp = true);
// issue the coalesced queued calls (rtg_render_async with no stream) not issued yet
int flush_pending(rtg_handle* h);
// the handle's stream waits for every queued chunk (called by every entry point that reads the film,
// the stats or slot 0's buffers, or synchronises)
int join_frames(rtg_handle* h);
// k_generate for the paths of a (camera rays at pixel centres, Scene.h:43-54)
int launch_generate(rtg_handle* h, const ChunkArgs& a, const PathBufs& pb, hipStream_t st);
// one k_trace launch (closest-hit rays of io.queue and any-hit rays of io.squeue) on stream st
// (max_blocks != 0: at most that many one-wave blocks instead of the resident grid)
int launch_trace(rtg_handle* h, const TraceIO& io, hipStream_t st, unsigned max_blocks = 0);
// rtg_shade.hip: one k_shade launch of `grid` blocks (ALT = alt, TAB = tab) for bounce b
int launch_shade(bool alt, bool tab, unsigned grid, hipStream_t st, const SceneView& s, const ChunkArgs& a,
                 const PathBufs& p, int b);
