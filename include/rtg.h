/*
 * rtg.h — C-ABI of the MI355X wavefront path tracer (librtg.so).
 *
 * This is the drop-in boundary for RTBase's per-pixel render loop. It replaces, one for one:
 *
 *   RayTracer::render()                 RTBase/Renderer.h:876-885  -> rtg_render()
 *     pathTracerTileBased/getTileID     RTBase/Renderer.h:820-853  (tile selection: tile_ids)
 *     renderTile                        RTBase/Renderer.h:795-818  (pixel centre rays, splat)
 *     pathTrace / computeDirect         RTBase/Renderer.h:328-392, 423-473
 *     Scene::traverse / Scene::visible  RTBase/Scene.h:107-130, 161-169
 *   Film::film / Film::SPP              RTBase/Imaging.h:201-261   -> rtg_film_*()
 *   Film::clear                         RTBase/Imaging.h:252-256   -> rtg_clear()
 *   Sampler::next (per-thread MTRandom) RTBase/Sampling.h:7-26     -> counter-based PCG32 stream
 *                                       keyed by (seed, pixel, sample)
 *
 * Everything above the boundary (scene.json/.gem loading, texture decode, BVH build with its
 * triangle permutation, light list, camera matrices, HDR writing) stays in the host; the host
 * hands over the *flattened reference Scene* below. No C++ or torch types cross this ABI.
 *
 * Conventions: 0 = success, negative = error (rtg_last_error() gives a message, thread-local).
 * A handle owns one GPU's copy of the scene and film; it is not thread-safe (one host thread
 * per handle). Inputs are copied during rtg_create; the caller may free them afterwards.
 */
#ifndef RTG_H
#define RTG_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: rtg_scene_desc.projection; 3: rtg_stats.tri_tail_loads / leafbox_tests appended;
 * 4: rtg_render_async queues frames (returns before any of its work has run), rtg_render_idle,
 *    rtg_stats.traced_camera_rays appended;
 * 5: rtg_build_id; the own-tile film exchange (rtg_tile_pixels, rtg_film_gather, rtg_film_scatter),
 *    which rtg_group_reduce now uses in place of a whole-film ncclReduce; rtg_stats.chunk_samples
 * 6: rtg_group_render_async / rtg_group_reduce_async / rtg_group_synchronize (queued group frames);
 *    rtg_film_scatter takes the film's pixel count; rtg_stats.lane_idle_* appended */
#define RTG_ABI_VERSION 6

/* error codes */
#define RTG_OK              0
#define RTG_ERR_ARG        -1
#define RTG_ERR_HIP        -2
#define RTG_ERR_NO_DEVICE  -3
#define RTG_ERR_NO_LIGHTS  -4
#define RTG_ERR_ALLOC      -5

/* Effective material kinds: RTBase has 8 BSDF classes but only three distinct
 * behaviours plus a pdf quirk. */
#define RTG_MAT_DIFFUSE   0  /* DiffuseBSDF             Materials.h:118-156 (pdf = z>=0 ? z/pi : 0)   */
#define RTG_MAT_LAMBERT   1  /* Conductor/Dielectric/OrenNayar/Plastic stubs (pdf = z/pi, no clamp)  */
#define RTG_MAT_MIRROR    2  /* MirrorBSDF              Materials.h:158-201                          */
#define RTG_MAT_GLASS     3  /* GlassBSDF               Materials.h:252-318 (one-sided)              */

typedef struct rtg_camera {        /* Camera, RTBase/Scene.h:10-70 */
    float inv_proj[16];            /* inverseProjectionMatrix.m (row-major)   */
    float camera[16];              /* camera.m (view -> world)                */
    float origin[3];               /* origin = camera.mulPoint(0,0,0)         */
    float width, height;           /* film size as the reference floats       */
} rtg_camera;

typedef struct rtg_camera_proj {   /* Camera members used by projectOntoCamera / connectToCamera   */
    float proj[16];                /* projectionMatrix.m (Scene.h:22-32, after the flipX negation)  */
    float camera_to_view[16];      /* cameraToView.m = camera.invert() (Scene.h:33-41)             */
    float view_direction[3];       /* viewDirection (Scene.h:38-40)                                */
    float a_film;                  /* Afilm = Wlens * Hlens (Scene.h:28-31)                         */
} rtg_camera_proj;

typedef struct rtg_material {      /* BSDF* + emission, RTBase/Materials.h:94-116 */
    int32_t kind;                  /* RTG_MAT_*                                    */
    int32_t two_sided;             /* BSDF::isTwoSided()                           */
    int32_t texture;               /* albedo Texture* as an index into textures    */
    float int_ior, ext_ior;        /* GlassBSDF::intIOR / extIOR (ignored otherwise) */
    float emission[3];             /* BSDF::emission (isLight iff Lum > 0)         */
} rtg_material;

typedef struct rtg_texture {       /* Texture, RTBase/Imaging.h:16-130 */
    int32_t width, height;
    const float* texels;           /* width*height*3, Colour r,g,b row-major */
} rtg_texture;

typedef struct rtg_scene_desc {    /* Scene after Scene::build(), RTBase/Scene.h:72-106 */
    uint32_t n_tris;               /* triangles in post-BVH-build order (Geometry.h:351 sort)  */
    const float* positions;        /* n_tris*9: vertices[0..2].p                               */
    const float* normals;          /* n_tris*9: vertices[0..2].normal                          */
    const float* uvs;              /* n_tris*6: (u,v) of vertices[0..2]                        */
    const uint32_t* material;      /* n_tris: Triangle::materialIndex                          */
    uint32_t n_nodes;              /* BVHNode tree flattened in DFS pre-order, root = 0        */
    const float* node_bounds;      /* n_nodes*6: bounds.min.xyz, bounds.max.xyz                */
    const int32_t* node_links;     /* n_nodes*4: l, r (-1 = none), startIndex, endIndex        */
    uint32_t n_materials;
    const rtg_material* materials;
    uint32_t n_textures;
    const rtg_texture* textures;
    int32_t env_texture;           /* -1: BackgroundColour(0,0,0); else EnvironmentMap(tex)    */
    uint32_t n_lights;             /* Scene::lights in order                                   */
    const int32_t* lights;         /* -1 = the environment light, else a triangle index        */
    rtg_camera camera;
    rtg_camera_proj projection;    /* light tracing / instant radiosity only (ABI version 2)   */
} rtg_scene_desc;

typedef struct rtg_stats {
    uint64_t paths;                /* camera paths traced                                      */
    uint64_t extension_rays;       /* closest-hit queries (Scene::traverse)                    */
    uint64_t shadow_rays;          /* any-hit queries (Scene::visible)                         */
    uint64_t node_visits;          /* RTG_OPT_COUNT: box tests by closest-hit rays             */
    uint64_t tri_tests;            /* RTG_OPT_COUNT: triangle tests by closest-hit rays        */
    uint64_t shadow_node_visits;   /* RTG_OPT_COUNT: box tests by any-hit rays                 */
    uint64_t shadow_tri_tests;     /* RTG_OPT_COUNT: triangle tests by any-hit rays            */
    uint64_t extend_launches;      /* RTG_OPT_TIMING: traversal launches in the last call      */
    double   render_ms;            /* device time of the last rtg_render call                  */
    double   extend_ms;            /* RTG_OPT_TIMING: traversal kernel time, extension + shadow */
                                   /* rays (one k_trace launch per bounce; last call)          */
    double   shadow_ms;            /* unused since shadow rays share the traversal launches (0) */
    double   shade_ms;             /* device time spent in generate/shade/accumulate kernels   */
    uint64_t lane_slots;           /* RTG_OPT_COUNT: closest-hit loop iterations x 64 lanes     */
    uint64_t node_lane_steps;      /* RTG_OPT_COUNT: lanes doing a node step, summed            */
    uint64_t leaf_lane_steps;      /* RTG_OPT_COUNT: lanes doing a leaf step, summed            */
    uint64_t leaf_phase_slots;     /* RTG_OPT_COUNT: leaf-phase iterations x 64 lanes           */
    uint64_t pops;                 /* RTG_OPT_COUNT: closest-hit stack pops                     */
    uint64_t cullable_pops;        /* RTG_OPT_COUNT: pops whose entry distance was > the hit    */
    uint64_t tri_tail_loads;       /* RTG_OPT_COUNT: triangle records whose last 16 B were fetched */
                                   /* (the plane distance was a candidate), all rays             */
    uint64_t leafbox_tests;        /* RTG_OPT_COUNT: reference leaf-box records fetched, all rays */
    uint64_t traced_camera_rays;   /* path tracer: camera rays traced. renderTile's camera ray is the   */
                                   /* pixel centre's for every sample (Renderer.h:805-808), so a chunk  */
                                   /* traces one per pixel and its samples share the first hit;         */
                                   /* extension_rays counts one per sample, as the reference casts them */
    uint64_t chunk_samples;        /* samples per pixel of the largest wavefront chunk issued since the */
                                   /* last rtg_clear (ABI 5): the chunk shape of the render           */
    /* RTG_OPT_COUNT (ABI 6): lanes not stepping a node in a traversal loop iteration, by reason,   */
    /* summed like node_lane_steps (lane_slots = node_lane_steps + these five)                      */
    uint64_t lane_idle_no_ray;       /* no ray: waiting for the wave's refill                        */
    uint64_t lane_idle_last_leaf;    /* walk done, its parked leaf waiting for the wave's leaf phase */
    uint64_t lane_idle_leaf_blocked; /* reached a leaf while its parked-leaf slots are full (two)    */
    uint64_t lane_idle_retiring;     /* ray finished, retired at the next iteration                  */
    uint64_t lane_idle_leaf_popped;  /* popped a leaf last iteration; parked in this one             */
} rtg_stats;

typedef struct rtg_handle rtg_handle;

int32_t     rtg_abi_version(void);
/* Hash of the sources, headers and compile flags this library was built from (build.py
 * source_hash("device")): a test or smoke run checks it against the tree it runs in. */
const char* rtg_build_id(void);
const char* rtg_last_error(void);
int         rtg_device_count(int* count);

/* Upload the scene to device `device` (HBM); allocates the film (width*height RGB float). */
int  rtg_create(int device, const rtg_scene_desc* desc, rtg_handle** out);
void rtg_destroy(rtg_handle* h);

/* Tracing options. max_depth is RTBase's MAX_DEPTH (Renderer.h:20, default 4): a path has at
 * most max_depth+2 closest-hit segments. flags: RTG_OPT_CULL enables the conservative distance
 * culling (without it traversal visits exactly the reference's node set: verification mode);
 * RTG_OPT_COUNT runs the counting kernels (node / triangle tests in rtg_stats);
 * RTG_OPT_TIMING records HIP events around every launch (per-kernel-class ms in rtg_stats; launches
 * of chunks running side by side in the frame pipeline each count their shared time);
 * RTG_OPT_BVH2 forces the reference BVH2 walk (no 4-wide collapse; verification / A-B).
 * max_paths_in_flight bounds the paths of one wavefront chunk (0 = keep, default 1G; a chunk's path
 * state is also held to half the free HBM). */
#define RTG_OPT_CULL   1
#define RTG_OPT_COUNT  2
#define RTG_OPT_TIMING 4
#define RTG_OPT_BVH2   8
#define RTG_OPT_WAVETIME 16  /* diagnostic builds only (RTG_DEBUG=1): per-wave clocks of k_trace on stderr */
#define RTG_OPT_SERIAL  32   /* one chunk in flight at a time, every k_shade grid sized from the live counts
                                read back during the traversal (verification / A-B of the frame pipeline) */
#define RTG_OPT_NO_COALESCE 64  /* queued calls (rtg_render_async, no stream) are issued one by one */
int  rtg_set_options(rtg_handle* h, int max_depth, int flags, uint32_t max_paths_in_flight);

/* Per-pixel estimator (the alternative RayTracer methods of Renderer.h). PATH is RayTracer::render's
 * pathTrace (Renderer.h:328-392, the default). DIRECT = RayTracer::direct (:393-407): emission or one
 * NEE sample at the first hit, 0 on a miss. ALBEDO = RayTracer::albedo (:558-571): emission,
 * BSDF::evaluate(sd, (0,1,0)) or the background. NORMALS = RayTracer::viewNormals (:572-582):
 * |shading normal| at the first hit. DIRECT_MIS = RayTracer::direct with computeDirectMIS
 * (:474-557) in place of computeDirect: one light sample and one BSDF sample combined by the
 * balance heuristic (the reference defines it but never calls it). */
#define RTG_INTEGRATOR_PATH       0
#define RTG_INTEGRATOR_DIRECT     1
#define RTG_INTEGRATOR_ALBEDO     2
#define RTG_INTEGRATOR_NORMALS    3
#define RTG_INTEGRATOR_DIRECT_MIS 4
int  rtg_set_integrator(rtg_handle* h, int integrator);

/* Add samples [first_sample, first_sample+n_samples) of every pixel in the listed 32x32 tiles
 * (tile id = ty*tilesX + tx, RTBase TILE_SIZE=32; tile_ids=NULL = all tiles) to the film, in
 * sample order per pixel. Equivalent to n_samples calls of RayTracer::render() with the
 * deterministic sampler.
 * rtg_render returns when the samples are on the film. rtg_render_async only queues them:
 *   - with hip_stream NULL it is the drop-in RayTracer::render() of a frame loop (Main.cpp:74-118):
 *     the call is queued and returns before its work starts. Consecutive queued calls with the same
 *     seed and tiles whose samples follow on (frame f, f+1, ...) are coalesced and issued together
 *     once 64M paths are pending (64 frames of a 1-Mpixel film), or as soon as anything reads the
 *     film or the stats, waits, or changes a setting (RTG_OPT_NO_COALESCE issues every call at
 *     once). Issued work of at most 16M paths per chunk runs in a pipeline of 3 slots, each with its
 *     own path state and stream, with no host wait: chunks run side by side on the GPU, a call waits
 *     only for the chunk three before it to leave the GPU, and the film updates stay in sample
 *     order, so the film is bit-identical to one rtg_render of all the samples. A pipelined chunk's
 *     traversal may start before the caller's earlier film reads on the handle (rtg_film_gather,
 *     ...) have run; only its film fold waits for them. Larger chunks (the
 *     call that reaches the 64M threshold issues one) read each bounce's live count back during the
 *     traversal, so that call returns once the chunk's last bounce is issued; the calls before it
 *     return at once. rtg_film_read with a film pointer,
 *     rtg_film_copy_device, rtg_get_stats, rtg_synchronize, rtg_render_idle, rtg_clear ... first
 *     issue and wait for the queued calls; rtg_film_read(h, NULL, &spp) returns Film::SPP at once.
 *     An error of a coalesced call is reported by the call that issues it.
 *   - with a hip_stream, the work is ordered after the caller's earlier work on that stream, and
 *     the caller's later work on it sees the film updated.
 * rtg_render_idle sets *idle to 1 when no queued render work is left on the GPU.
 * Sample indices must stay below RTG_MAX_SAMPLES_PER_KEY: the PCG stream of (pixel, sample) is
 * keyed seq = pixel << 16 | sample; more samples take another seed. */
#define RTG_MAX_SAMPLES_PER_KEY 65536u
int  rtg_render(rtg_handle* h, uint32_t first_sample, uint32_t n_samples, uint64_t seed,
                const uint32_t* tile_ids, uint32_t n_tiles);
int  rtg_render_async(rtg_handle* h, uint32_t first_sample, uint32_t n_samples, uint64_t seed,
                      const uint32_t* tile_ids, uint32_t n_tiles, void* hip_stream);
int  rtg_synchronize(rtg_handle* h);
int  rtg_render_idle(rtg_handle* h, int* idle);

/* RayTracer::adaptiveRender (Renderer.h:583-749), one frame (Film::SPP += 1). Pass 1 renders
 * init_samples samples of every pixel (sample indices first_sample ...) into a scratch film and
 * takes each 32x32 tile's variance of the per-pixel means (adaptiveSampling, :583-638); a tile's
 * weight is its share of the total variance; pass 2 renders max((int)(sqrt(weight) * max_samples),
 * min_samples) samples of each pixel of the tile (indices first_sample + init_samples ...) and adds
 * their mean to the film (sampleTileWithWeight, :640-672). The reference constants are INIT_SAMPLES
 * 2, MAX_SAMPLES 10240, MIN_SAMPLES 1 (Renderer.h:20-23). tile_samples (optional, tilesX*tilesY)
 * receives each tile's pass-2 sample count. first_sample + init_samples + the largest tile count
 * must be <= RTG_MAX_SAMPLES_PER_KEY (checked before the film is touched: RTG_ERR_ARG). Pass 2 is
 * staged and published only when every tile group succeeded, so a failed call leaves the film and
 * SPP as they were. */
/* RayTracer::lightTracer (Renderer.h:221-326): each frame traces width*height light paths (path i
 * of frame f draws from the PCG stream keyed (seed, i, f)), connects every non-specular vertex to
 * the camera (connectToCamera: projectOntoCamera, importance W_e = 1/(Afilm cos^4), visibility)
 * and splats the result into the film in (path, vertex) order per pixel, as the reference's
 * single-threaded loop does. Film::SPP += 1 per frame. The film must have < 2^24 pixels. */
int  rtg_render_light(rtg_handle* h, uint32_t first_frame, uint32_t n_frames, uint64_t seed);
/* RayTracer::instantRadiosity (Renderer.h:82-218): each frame traces n_vpl_paths VPL paths
 * (traceVPLs; the reference uses MAX_VPL = 50) and then, for every pixel whose camera ray hits a
 * surface, sums vpl.Le * BSDF * G over every visible VPL in VPL order (computeVPLsContribution)
 * and splats it. Film::SPP += 1 per frame. */
#define RTG_MAX_VPL 50
int  rtg_render_instant_radiosity(rtg_handle* h, uint32_t first_frame, uint32_t n_frames, uint64_t seed,
                                  uint32_t n_vpl_paths);

#define RTG_ADAPTIVE_INIT_SAMPLES 2
#define RTG_ADAPTIVE_MAX_SAMPLES  10240
#define RTG_ADAPTIVE_MIN_SAMPLES  1
int  rtg_render_adaptive(rtg_handle* h, uint32_t first_sample, uint64_t seed, uint32_t init_samples,
                         uint32_t max_samples, uint32_t min_samples, uint32_t* tile_samples);

/* ---- one node, several GPUs (rtg_multi.hip). RayTracer::pathTracerTileBased spreads 32x32 tiles
 * over numProcs CPU threads (Renderer.h:836-853, numProcs from :52-54); here the tiles are spread
 * over devices: rank r of N renders every sample of the tiles with (tile_x + tile_y) % N == r
 * (rtg_tiles_for_rank; the partition of raytracingrenderer_amd/distributed.py), one host thread and
 * one handle per device, and rtg_group_reduce assembles the film on devices[0] from each rank's own
 * tiles only: every rank packs its tiles' pixels (rtg_film_gather), sends them to devices[0] with
 * one ncclSend (ncclCommInitAll, single process; devices[0] posts an ncclRecv per rank), and
 * devices[0] scatters them into the film (rtg_film_scatter). Tile supports are disjoint and cover
 * the image, so the assembled film is bit-identical to a one-device render (and to the sum of the
 * films), at 1/N of a whole-film reduce's bytes per rank. A device list with repeats (N ranks
 * rehearsed on fewer GPUs) renders the ranks in turn and moves the packed tiles with device copies.
 * The scene's device records are built on the host once and uploaded to the devices in parallel
 * (rtg_group_setup_ms). A failed rtg_group_render leaves the group poisoned (other ranks already
 * added their samples): rtg_group_reduce / film_read return RTG_ERR_ARG until rtg_group_clear. */
typedef struct rtg_group rtg_group;
int  rtg_tiles_for_rank(uint32_t width, uint32_t height, int rank, int world, uint32_t* tile_ids /* or NULL */,
                        uint32_t* n_tiles);
int  rtg_group_create(const int* devices, int n_devices, const rtg_scene_desc* desc, rtg_group** out);
void rtg_group_destroy(rtg_group* g);
int  rtg_group_size(rtg_group* g);
rtg_handle* rtg_group_handle(rtg_group* g, int rank);  /* e.g. for rtg_get_stats; owned by the group */
int  rtg_group_set_options(rtg_group* g, int max_depth, int flags, uint32_t max_paths);
int  rtg_group_render(rtg_group* g, uint32_t first_sample, uint32_t n_samples, uint64_t seed);
int  rtg_group_reduce(rtg_group* g);  /* the films stay per device; the assembled film goes to a separate buffer */
/* Queued forms (the frame loop of Main.cpp:74-118 on N devices). rtg_group_render_async is every
 * rank's rtg_render_async (NULL stream) on its device: frames are coalesced and pipelined per rank
 * as on one handle, and the call returns without waiting for the GPUs. rtg_group_reduce_async
 * queues the own-tile exchange on per-rank exchange streams after each rank's queued frames (pack,
 * RCCL send/recv, scatter on devices[0]); the ranks' next frames start their traversal meanwhile
 * and only their film folds wait for the packs. rtg_group_synchronize waits for both;
 * rtg_group_film_read waits for the exchange it reads. */
int  rtg_group_render_async(rtg_group* g, uint32_t first_sample, uint32_t n_samples, uint64_t seed);
int  rtg_group_reduce_async(rtg_group* g);
int  rtg_group_synchronize(rtg_group* g);
int  rtg_group_film_read(rtg_group* g, float* rgb_sum /* width*height*3 */, uint32_t* spp);  /* reduces if needed */
int  rtg_group_clear(rtg_group* g);
double rtg_group_reduce_ms(rtg_group* g);  /* device time of the last reduce (set when the group is synchronized) */
int  rtg_group_uses_rccl(rtg_group* g);    /* 1: RCCL communicator; 0: device copies (repeated devices) or one
                                              device (no communicator unless RTG_GROUP_RCCL1=1 is set) */
int  rtg_group_setup_ms(rtg_group* g, double* prepare_ms, double* upload_ms);  /* host build, parallel uploads */

/* ---- own-tile film exchange (the data movement of rtg_group_reduce, exposed for hosts that run
 * one process per GPU, e.g. raytracingrenderer_amd/distributed.py over torch.distributed).
 * rtg_tile_pixels lists the film pixel indices (y * width + x) of the given 32x32 tiles in the
 * order rtg_film_gather packs them: tile by tile, row-major inside a tile, clipped at the film
 * edge (pixels NULL: only the count). rtg_film_gather copies the handle's film pixels listed in
 * pixels_dev (device array of n indices; 0xFFFFFFFF = padding, packed as zeros) to dst_dev (3n
 * floats), ordered after every render queued on the handle, and the handle's later film writes
 * (the folds of renders queued after it) wait for it; rtg_film_scatter writes src_dev's n
 * packed pixels into film_dev (film_pixels * 3 floats) at the listed indices (0xFFFFFFFF:
 * skipped). An index at or past the film's pixel count is treated as padding by both (never
 * read or written). Both run on hip_stream (NULL: the handle's stream / the device's null stream) and
 * return without waiting. */
int  rtg_tile_pixels(uint32_t width, uint32_t height, const uint32_t* tile_ids, uint32_t n_tiles,
                     uint32_t* pixels /* or NULL */, uint32_t* n_pixels);
int  rtg_film_gather(rtg_handle* h, const uint32_t* pixels_dev, uint32_t n, float* dst_dev, void* hip_stream);
int  rtg_film_scatter(int device, const float* src_dev, const uint32_t* pixels_dev, uint32_t n, float* film_dev,
                      uint32_t film_pixels /* width * height of film_dev */, void* hip_stream);

/* Film access: the unnormalised sum (Film::film) and the sample count (Film::SPP). */
int  rtg_film_read(rtg_handle* h, float* rgb_sum /* width*height*3 */, uint32_t* spp);
int  rtg_film_copy_device(rtg_handle* h, void* dst_device /* width*height*3 floats */);
int  rtg_film_load(rtg_handle* h, const float* rgb_sum, uint32_t spp);  /* resume */
int  rtg_clear(rtg_handle* h);
int  rtg_get_stats(rtg_handle* h, rtg_stats* out);
/* Per traversal launch (k_trace) device time of the last render with RTG_OPT_TIMING, in launch
 * order (chunk by chunk, bounce by bounce): n receives the count, at most max are written. */
int  rtg_launch_times(rtg_handle* h, double* trace_ms, uint32_t max, uint32_t* n);
/* The rays each trace launch of the last timed render's last chunk walked (path tracer: launch b =
 * bounce b's extension rays + bounce b-1's shadow rays; launch 0 the camera rays, one per pixel). */
int  rtg_launch_rays(rtg_handle* h, uint64_t* rays, uint32_t max, uint32_t* n);
/* Diagnostics of the locality-matched roofline (builds with RTG_DEBUG=1 only; RTG_ERR_ARG
 * otherwise). rtg_debug_capture(h, b): the next render records every record fetch of trace launch
 * b of its first chunk, per ray in order (-1: off). rtg_debug_replay(h, out[4]) replays that
 * stream (same addresses, order, grouping and occupancy; nothing but the fetches and 64 VALU per
 * step) on the device: out = {best of 3 replay ms, fetches, extension rays, shadow rays}. */
int  rtg_debug_capture(rtg_handle* h, int launch);
int  rtg_debug_replay(rtg_handle* h, double* out);

/* Low-level ray queries on the uploaded scene (test / oracle comparison surface).
 * rays: n*8 floats (o.xyz, tmax, dir.xyz, pad). For closest-hit, tmax is ignored and the result
 * is n*4 (t, id-as-float-bits, alpha, beta) with t = FLT_MAX on miss (IntersectionData,
 * Geometry.h:231-238). For any-hit, tmax is Scene::visible's maxT and the result is n int32
 * (1 = visible). Device-side arrays are allocated internally; inputs are host pointers. */
int  rtg_trace_closest(rtg_handle* h, const float* rays, uint32_t n, float* hits);
/* BSDF::sample / evaluate probe on the current device (Materials.h:118-318), scripted draws.
 * cases: n*20 floats (kind, int_ior, ext_ior, albedo.rgb of a 1x1 texture, sNormal.xyz, wo.xyz,
 * tu, tv, draw[4], pad[2]);
 * out: n*11 floats (wi.xyz, reflectedColour.rgb, pdf, draws consumed, evaluate(wi).rgb). */
int  rtg_probe_bsdf(const float* cases, uint32_t n, float* out);
int  rtg_trace_visible(rtg_handle* h, const float* rays, uint32_t n, int32_t* visible);
/* Transcendental probe on the current device: the kernels' acosf / sinf / cosf / atan2f
 * (include/rtg_math.h, the reference platform's glibc restated; RTBase/Sampling.h:35-61,
 * Core.h:549-557, Lights.h:152-155) on n inputs. fn: RTG_MATH_SINF, _COSF, _SINCOSF (out 2n:
 * sin, cos), _ACOSF, _ATAN2F (in 2n: y, x). n < 2^31. */
#define RTG_MATH_SINF   0
#define RTG_MATH_COSF   1
#define RTG_MATH_SINCOSF 2
#define RTG_MATH_ACOSF  3
#define RTG_MATH_ATAN2F 4
int  rtg_probe_math(int fn, const float* in, uint32_t n, float* out);

#ifdef __cplusplus
}
#endif
#endif /* RTG_H */
