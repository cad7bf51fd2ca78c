// rtg_multi.hip — one-node multi-GPU rendering behind the C-ABI (include/rtg.h, rtg_group_*), and
// the own-tile film exchange (rtg_tile_pixels / rtg_film_gather / rtg_film_scatter).
//
// RTBase's only parallelism is the tile pool of RayTracer::pathTracerTileBased (Renderer.h:836-853:
// numProcs threads pop 32x32 tiles from a shared queue, Renderer.h:52-54). Here the tiles are
// spread over the GPUs of one node instead: device r renders every sample of the tiles with
// (tile_x + tile_y) % N == r (diagonal stripes, the same partition as raytracingrenderer_amd/
// distributed.py), one host thread and one rtg_handle per device. The film is then assembled on
// the first device from each rank's own tiles: rank r packs the pixels of its tiles (k_film_gather,
// 12 B per pixel: 1/N of the film), sends them with one ncclSend over xGMI (ncclCommInitAll over
// the devices, single process; the first device posts one ncclRecv per rank inside the same RCCL
// group), and the first device scatters every rank's pixels into the film (k_film_scatter). Tile
// supports are disjoint and cover the image, so the assembled film is the one-GPU film bit for
// bit. (Until round 4 every rank sent its whole film to an ncclReduce: N x the bytes, 7/8 of them
// +0.0 at N = 8.)
//
// A device list that repeats a device (rehearsing N ranks on one GPU) cannot form an RCCL
// communicator; the ranks then render one after another, each with an equal share of the device's
// memory for its chunks (rtg_handle::mem_cap), and the packed tiles move with device copies into
// the same receive buffer and scatter as the RCCL path.
//
// Setup: the scene's device records are built once on the host (prepare_scene: triangle records,
// the wide tree over the reference leaves, leaf boxes, materials, textures) and uploaded to every
// device by its own thread (upload_scene), so an 8-GPU group costs one host build, not eight.
// A rank that fails a render poisons the group: the other ranks' films already hold the samples,
// so reduce / film_read refuse until rtg_group_clear.
//
// RCCL is opened with dlopen when a group first needs a communicator (not linked into librtg):
// a process that also loads PyTorch gets PyTorch's bundled RCCL (same soname) instead of a second
// copy, and librtg never pulls RCCL into processes that do not use groups.
#include "rtg_internal.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {
struct Rccl {
    bool tried = false, ok = false;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};
Rccl g_rccl;
std::mutex g_rccl_mu;

bool load_rccl() {
    std::lock_guard<std::mutex> lock(g_rccl_mu);
    if (g_rccl.tried) return g_rccl.ok;
    g_rccl.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        g_err = std::string("RCCL not found: ") + dlerror();
        return false;
    }
    g_rccl.comm_init_all = (decltype(g_rccl.comm_init_all))dlsym(h, "ncclCommInitAll");
    g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))dlsym(h, "ncclCommDestroy");
    g_rccl.send = (decltype(g_rccl.send))dlsym(h, "ncclSend");
    g_rccl.recv = (decltype(g_rccl.recv))dlsym(h, "ncclRecv");
    g_rccl.group_start = (decltype(g_rccl.group_start))dlsym(h, "ncclGroupStart");
    g_rccl.group_end = (decltype(g_rccl.group_end))dlsym(h, "ncclGroupEnd");
    g_rccl.error_string = (decltype(g_rccl.error_string))dlsym(h, "ncclGetErrorString");
    g_rccl.ok = g_rccl.comm_init_all && g_rccl.comm_destroy && g_rccl.send && g_rccl.recv && g_rccl.group_start &&
                g_rccl.group_end && g_rccl.error_string;
    if (!g_rccl.ok) g_err = "RCCL: missing symbols";
    return g_rccl.ok;
}

}  // namespace

// Own-tile film exchange. Pack: dst[i] = film[pix[i]] (3 floats; a padding index packs zeros).
// Scatter: film[pix[i]] = src[i] (padding skipped). One thread per pixel, 12-B reads and writes:
// HBM-bound, 24 B per pixel moved.
#define RTG_PIX_PAD 0xFFFFFFFFu
// An index at or past the film's pixel count (a list built for another film size) is treated as
// padding: packed as zeros, skipped by the scatter, never dereferenced.
__global__ __launch_bounds__(256) void k_film_gather(const float* __restrict__ film, const uint32_t* __restrict__ pix,
                                                     uint32_t n, uint32_t film_pixels, float* __restrict__ dst) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = pix[i];
    float r = 0.0f, g = 0.0f, b = 0.0f;
    if (p < film_pixels) {
        r = film[3 * (size_t)p];
        g = film[3 * (size_t)p + 1];
        b = film[3 * (size_t)p + 2];
    }
    dst[3 * (size_t)i] = r;
    dst[3 * (size_t)i + 1] = g;
    dst[3 * (size_t)i + 2] = b;
}

__global__ __launch_bounds__(256) void k_film_scatter(const float* __restrict__ src, const uint32_t* __restrict__ pix,
                                                      uint32_t n, uint32_t film_pixels, float* __restrict__ film) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = pix[i];
    if (p >= film_pixels) return;  // padding (RTG_PIX_PAD) or out of range
    film[3 * (size_t)p] = src[3 * (size_t)i];
    film[3 * (size_t)p + 1] = src[3 * (size_t)i + 1];
    film[3 * (size_t)p + 2] = src[3 * (size_t)i + 2];
}

// the pixel order of set_pixels (rtg_kernels.hip): tile by tile, row-major inside a tile
static void tile_pixels(uint32_t W, uint32_t H, const uint32_t* tiles, uint32_t n_tiles, std::vector<uint32_t>& out) {
    const uint32_t tx = (W + 31) / 32;
    for (uint32_t i = 0; i < n_tiles; ++i) {
        const uint32_t bx = (tiles[i] % tx) * 32, by = (tiles[i] / tx) * 32;
        for (uint32_t y = by; y < std::min<uint32_t>(by + 32, H); ++y)
            for (uint32_t x = bx; x < std::min<uint32_t>(bx + 32, W); ++x) out.push_back(y * W + x);
    }
}

struct rtg_group {
    std::vector<int> devices;
    std::vector<rtg_handle*> h;
    std::vector<std::vector<uint32_t>> tiles;  // per rank
    std::vector<ncclComm_t> comms;             // empty: device copies (repeated devices)
    float* d_sum = nullptr;                    // assembled film on devices[0]
    // own-tile exchange: rank r's pixel list and pack buffer on its device (npix[r] pixels); on
    // devices[0] the receive buffer (rank r's pixels at r * maxpix) and the matching pixel lists
    std::vector<uint32_t*> d_pix;
    std::vector<float*> d_pack;
    std::vector<uint32_t> npix;
    uint32_t maxpix = 0;
    uint32_t* d_pix_all = nullptr;
    float* d_recv = nullptr;
    uint32_t W = 0, H = 0;
    uint32_t reduced_spp = 0;
    bool reduced = false;
    bool distinct = true;                      // every rank on its own device (RCCL, concurrent ranks)
    bool poisoned = false;                     // a rank failed a render: films hold partial samples
    double reduce_ms = 0.0;
    double prepare_ms = 0.0, upload_ms = 0.0;  // group setup: host build once, parallel uploads
    // the exchange's own streams, one per rank on its device (rank r: its pack and send; devices[0]
    // also the receives and the scatter), so that a queued exchange (rtg_group_reduce_async) runs
    // beside the ranks' next frames instead of in their render streams
    std::vector<hipStream_t> xs;
    std::vector<hipEvent_t> xpacked;           // repeated devices: rank r's pack is done
    hipEvent_t xcopied = nullptr;              // repeated devices: devices[0] has copied every pack
    hipEvent_t xe0 = nullptr, xe1 = nullptr;   // devices[0]: rank 0's frames on its film / scatter done
    bool xtimed = false;                       // xe0 / xe1 hold an exchange not yet read into reduce_ms
    // (test mode, RTG_GROUP_RCCL_SELF=1 with a communicator) rank 0 also sends its pack to itself
    // with ncclSend / ncclRecv, so the RCCL exchange's calls run on a one-GPU box
    bool rccl_self = false;
};

// the own-tile exchange's buffers: per rank its pixel list + pack buffer on its device, on devices[0]
// a receive buffer of N x maxpix pixels and the concatenated (padded) pixel lists
static int exchange_setup(rtg_group* g) {
    const size_t n = g->h.size();
    std::vector<std::vector<uint32_t>> pl(n);
    for (size_t r = 0; r < n; ++r) {
        tile_pixels(g->W, g->H, g->tiles[r].data(), (uint32_t)g->tiles[r].size(), pl[r]);
        g->npix.push_back((uint32_t)pl[r].size());
        g->maxpix = std::max(g->maxpix, (uint32_t)pl[r].size());
    }
    const size_t mp = std::max<uint32_t>(g->maxpix, 1);
    std::vector<uint32_t> all(n * mp, RTG_PIX_PAD);
    for (size_t r = 0; r < n; ++r) std::copy(pl[r].begin(), pl[r].end(), all.begin() + r * mp);
    HIPOK(hipSetDevice(g->devices[0]));
    HIPOK(hipMalloc((void**)&g->d_recv, n * mp * 3 * sizeof(float)));
    if (dev_upload(&g->d_pix_all, all)) return RTG_ERR_HIP;
    HIPOK(hipEventCreate(&g->xe0));
    HIPOK(hipEventCreate(&g->xe1));
    HIPOK(hipEventCreateWithFlags(&g->xcopied, hipEventDisableTiming));
    g->d_pix.assign(n, nullptr);
    g->d_pack.assign(n, nullptr);
    g->xs.assign(n, nullptr);
    g->xpacked.assign(n, nullptr);
    for (size_t r = 0; r < n; ++r) {
        HIPOK(hipSetDevice(g->devices[r]));
        if (dev_upload(&g->d_pix[r], pl[r])) return RTG_ERR_HIP;
        if (r == 0 && !g->rccl_self) g->d_pack[r] = g->d_recv;
        else HIPOK(hipMalloc((void**)&g->d_pack[r], mp * 3 * sizeof(float)));
        HIPOK(hipStreamCreateWithFlags(&g->xs[r], hipStreamNonBlocking));
        HIPOK(hipEventCreateWithFlags(&g->xpacked[r], hipEventDisableTiming));
    }
    return RTG_OK;
}

// Runs fn(r) for every rank: one host thread per rank when every rank has a device of its own (a
// rank's call may wait on the host: back-pressure of the frame pipeline, a big chunk's count
// read-backs), in turn otherwise. The first failing rank's code is returned and the group poisoned.
template <class F>
static int for_ranks(rtg_group* g, F fn) {
    const size_t n = g->h.size();
    std::vector<int> rc(n, RTG_OK);
    std::vector<std::string> err(n);
    auto run = [&](size_t r) {
        rc[r] = fn(r);
        if (rc[r]) err[r] = rtg_last_error();  // g_err is thread-local
    };
    if (n == 1 || !g->distinct) {
        for (size_t r = 0; r < n; ++r) run(r);
    } else {
        std::vector<std::thread> pool;
        for (size_t r = 0; r < n; ++r) pool.emplace_back(run, r);
        for (auto& t : pool) t.join();
    }
    for (size_t r = 0; r < n; ++r)
        if (rc[r]) {
            g->poisoned = true;
            g_err = "rank " + std::to_string(r) + ": " + err[r] + " (group films now partial: rtg_group_clear)";
            return rc[r];
        }
    return RTG_OK;
}

// every rank's queued frames and the queued exchanges have finished; the last exchange's device time
// goes to reduce_ms
static int group_sync(rtg_group* g) {
    for (size_t r = 0; r < g->h.size(); ++r) {
        if (int rc = rtg_synchronize(g->h[r])) return rc;
        HIPOK(hipSetDevice(g->devices[r]));
        if (r < g->xs.size() && g->xs[r]) HIPOK(hipStreamSynchronize(g->xs[r]));
    }
    if (g->xtimed) {
        float ms = 0.0f;
        HIPOK(hipSetDevice(g->devices[0]));
        if (hipEventElapsedTime(&ms, g->xe0, g->xe1) == hipSuccess) g->reduce_ms = ms;
        g->xtimed = false;
    }
    return RTG_OK;
}

extern "C" {

int rtg_tile_pixels(uint32_t width, uint32_t height, const uint32_t* tile_ids, uint32_t n_tiles, uint32_t* pixels,
                    uint32_t* n_pixels) {
    if (!n_pixels || (!tile_ids && n_tiles)) {
        g_err = "rtg_tile_pixels: bad argument";
        return RTG_ERR_ARG;
    }
    const uint32_t nt = ((width + 31) / 32) * ((height + 31) / 32);
    for (uint32_t i = 0; i < n_tiles; ++i)
        if (tile_ids[i] >= nt) {
            g_err = "rtg_tile_pixels: tile id out of range";
            return RTG_ERR_ARG;
        }
    std::vector<uint32_t> pl;
    tile_pixels(width, height, tile_ids, n_tiles, pl);
    *n_pixels = (uint32_t)pl.size();
    if (pixels) std::copy(pl.begin(), pl.end(), pixels);
    return RTG_OK;
}

int rtg_film_gather(rtg_handle* h, const uint32_t* pixels_dev, uint32_t n, float* dst_dev, void* stream) {
    if (!h || (n && (!pixels_dev || !dst_dev))) {
        g_err = "rtg_film_gather: bad argument";
        return RTG_ERR_ARG;
    }
    HIPOK(hipSetDevice(h->device));
    if (int rc = join_frames(h)) return rc;  // the film holds every queued frame first
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    if (st != h->stream) {
        HIPOK(hipEventRecord(h->ev[2], h->stream));
        HIPOK(hipStreamWaitEvent(st, h->ev[2], 0));
    }
    if (n) {
        hipLaunchKernelGGL(k_film_gather, dim3((n + 255) / 256), dim3(256), 0, st, (const float*)h->d_film, pixels_dev, n,
                           (uint32_t)h->W * (uint32_t)h->H, dst_dev);
        LAUNCH_OK("k_film_gather");
        if (st != h->stream) {
            // the handle's later film writes (the next renders' folds wait on its stream) come after
            // this read of the film
            HIPOK(hipEventRecord(h->ev[3], st));
            HIPOK(hipStreamWaitEvent(h->stream, h->ev[3], 0));
        }
    }
    return RTG_OK;
}

int rtg_film_scatter(int device, const float* src_dev, const uint32_t* pixels_dev, uint32_t n, float* film_dev,
                     uint32_t film_pixels, void* stream) {
    if (n && (!src_dev || !pixels_dev || !film_dev || !film_pixels)) {
        g_err = "rtg_film_scatter: bad argument";
        return RTG_ERR_ARG;
    }
    HIPOK(hipSetDevice(device));
    if (n) {
        hipLaunchKernelGGL(k_film_scatter, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, src_dev, pixels_dev,
                           n, film_pixels, film_dev);
        LAUNCH_OK("k_film_scatter");
    }
    return RTG_OK;
}

int rtg_tiles_for_rank(uint32_t width, uint32_t height, int rank, int world, uint32_t* tile_ids, uint32_t* n_tiles) {
    if (!n_tiles || world < 1 || rank < 0 || rank >= world) {
        g_err = "rtg_tiles_for_rank: bad argument";
        return RTG_ERR_ARG;
    }
    const uint32_t tx = (width + 31) / 32, ty = (height + 31) / 32;
    uint32_t n = 0;
    for (uint32_t t = 0; t < tx * ty; ++t)
        if (((t % tx) + (t / tx)) % (uint32_t)world == (uint32_t)rank) {
            if (tile_ids) tile_ids[n] = t;
            ++n;
        }
    *n_tiles = n;
    return RTG_OK;
}

void rtg_group_destroy(rtg_group* g) {
    if (!g) return;
    (void)group_sync(g);  // queued frames and exchanges still use the buffers
    for (ncclComm_t c : g->comms) (void)g_rccl.comm_destroy(c);
    for (size_t r = 0; r < g->d_pix.size(); ++r) {
        (void)hipSetDevice(g->devices[r]);
        (void)hipFree(g->d_pix[r]);
        if (r > 0 || g->rccl_self) (void)hipFree(g->d_pack[r]);  // rank 0 packs straight into d_recv
        if (r < g->xs.size() && g->xs[r]) (void)hipStreamDestroy(g->xs[r]);
        if (r < g->xpacked.size() && g->xpacked[r]) (void)hipEventDestroy(g->xpacked[r]);
    }
    if (!g->devices.empty()) {
        (void)hipSetDevice(g->devices[0]);
        (void)hipFree(g->d_sum);
        (void)hipFree(g->d_recv);
        (void)hipFree(g->d_pix_all);
        if (g->xe0) (void)hipEventDestroy(g->xe0);
        if (g->xe1) (void)hipEventDestroy(g->xe1);
        if (g->xcopied) (void)hipEventDestroy(g->xcopied);
    }
    for (rtg_handle* h : g->h) rtg_destroy(h);
    delete g;
}

int rtg_group_create(const int* devices, int n_devices, const rtg_scene_desc* desc, rtg_group** out) {
    if (!devices || n_devices < 1 || !desc || !out) {
        g_err = "rtg_group_create: bad argument";
        return RTG_ERR_ARG;
    }
    *out = nullptr;
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc) return rc;
    auto t1 = clk::now();
    rtg_group* g = new rtg_group();
    g->devices.assign(devices, devices + n_devices);
    g->W = desc->camera.width;
    g->H = desc->camera.height;
    g->prepare_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    g->h.assign(n_devices, nullptr);
    std::vector<int> rcs(n_devices, RTG_OK);
    std::vector<std::string> errs(n_devices);
    auto up = [&](int r) {
        rtg_handle* h = new rtg_handle();
        rcs[r] = upload_scene(devices[r], hs, h);
        if (rcs[r]) {
            errs[r] = g_err;  // thread-local
            rtg_destroy(h);
            return;
        }
        g->h[r] = h;
    };
    {
        std::vector<std::thread> pool;
        for (int r = 0; r < n_devices; ++r) pool.emplace_back(up, r);
        for (auto& t : pool) t.join();
    }
    g->upload_ms = std::chrono::duration<double, std::milli>(clk::now() - t1).count();
    for (int r = 0; r < n_devices; ++r)
        if (rcs[r]) {
            rc = rcs[r];
            g_err = "rank " + std::to_string(r) + ": " + errs[r];
            g->h.erase(std::remove(g->h.begin(), g->h.end(), nullptr), g->h.end());
            rtg_group_destroy(g);
            return rc;
        }
    for (int r = 0; r < n_devices; ++r) {
        uint32_t n = 0;
        rtg_tiles_for_rank(g->W, g->H, r, n_devices, nullptr, &n);
        g->tiles.emplace_back(n);
        rtg_tiles_for_rank(g->W, g->H, r, n_devices, g->tiles.back().data(), &n);
    }
    std::vector<int> sorted(g->devices);
    std::sort(sorted.begin(), sorted.end());
    g->distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (!g->distinct) {
        // ranks rehearsed on one device render in turn, each keeping its chunk buffers: give each
        // an equal share of half the device's free HBM, so every rank runs the same chunk sizes
        // (left to the free-memory reading, later ranks got ever smaller chunks)
        for (int r = 0; r < n_devices; ++r) {
            const int k = (int)std::count(g->devices.begin(), g->devices.end(), g->devices[r]);
            size_t freeb = 0, totalb = 0;
            if (hipSetDevice(g->devices[r]) == hipSuccess && hipMemGetInfo(&freeb, &totalb) == hipSuccess)
                g->h[r]->mem_cap = std::max<size_t>(1, freeb / 2 / (size_t)k);
        }
    }
    // A group of one device has nothing to exchange and forms no communicator: an RCCL communicator in
    // the process slowed the renders by ~2 % (k_accumulate_pm 1.05 -> 1.52 ms per 64M-path fold,
    // DESIGN.md §7). RTG_GROUP_RCCL1=1 forms one anyway (the tests of the RCCL setup on a 1-GPU box).
    if (g->distinct && (n_devices > 1 || std::getenv("RTG_GROUP_RCCL1"))) {
        if (!load_rccl()) {
            rtg_group_destroy(g);
            return RTG_ERR_HIP;
        }
        g->comms.resize(n_devices);
        const ncclResult_t nr = g_rccl.comm_init_all(g->comms.data(), n_devices, g->devices.data());
        if (nr != ncclSuccess) {
            g->comms.clear();
            g_err = std::string("ncclCommInitAll: ") + g_rccl.error_string(nr);
            rtg_group_destroy(g);
            return RTG_ERR_HIP;
        }
    }
    g->rccl_self = !g->comms.empty() && std::getenv("RTG_GROUP_RCCL_SELF") != nullptr;
    if (hipSetDevice(g->devices[0]) != hipSuccess ||
        hipMalloc((void**)&g->d_sum, (size_t)g->W * g->H * 3 * sizeof(float)) != hipSuccess) {
        g_err = "rtg_group_create: film allocation failed";
        rtg_group_destroy(g);
        return RTG_ERR_HIP;
    }
    if (int rc2 = exchange_setup(g)) {
        rtg_group_destroy(g);
        return rc2;
    }
    *out = g;
    return RTG_OK;
}

int rtg_group_setup_ms(rtg_group* g, double* prepare_ms, double* upload_ms) {
    if (!g) return RTG_ERR_ARG;
    if (prepare_ms) *prepare_ms = g->prepare_ms;
    if (upload_ms) *upload_ms = g->upload_ms;
    return RTG_OK;
}

int rtg_group_size(rtg_group* g) { return g ? (int)g->h.size() : 0; }

rtg_handle* rtg_group_handle(rtg_group* g, int rank) {
    return (g && rank >= 0 && rank < (int)g->h.size()) ? g->h[rank] : nullptr;
}

int rtg_group_set_options(rtg_group* g, int max_depth, int flags, uint32_t max_paths) {
    if (!g) return RTG_ERR_ARG;
    for (rtg_handle* h : g->h) {
        const int rc = rtg_set_options(h, max_depth, flags, max_paths);
        if (rc) return rc;
    }
    return RTG_OK;
}

int rtg_group_render(rtg_group* g, uint32_t first_sample, uint32_t n_samples, uint64_t seed) {
    if (!g) return RTG_ERR_ARG;
    g->reduced = false;
    return for_ranks(g, [&](size_t r) {
        const std::vector<uint32_t>& t = g->tiles[r];
        if (t.empty()) return (int)RTG_OK;  // more devices than tiles: this rank's film stays zero
        return rtg_render(g->h[r], first_sample, n_samples, seed, t.data(), (uint32_t)t.size());
    });
}

// The queued frame of a group (the frame loop of Main.cpp:74-118 on N devices): every rank's
// rtg_render_async on its own device, so the ranks' frames are coalesced and pipelined exactly as one
// handle's are, and the call returns without waiting for the GPUs (a rank's call waits only for the
// frame pipeline's back-pressure or a big chunk's count read-backs, on its own host thread).
int rtg_group_render_async(rtg_group* g, uint32_t first_sample, uint32_t n_samples, uint64_t seed) {
    if (!g) return RTG_ERR_ARG;
    g->reduced = false;
    return for_ranks(g, [&](size_t r) {
        const std::vector<uint32_t>& t = g->tiles[r];
        if (t.empty()) return (int)RTG_OK;
        return rtg_render_async(g->h[r], first_sample, n_samples, seed, t.data(), (uint32_t)t.size(), nullptr);
    });
}

// The own-tile exchange, queued on the exchange streams (xs): rank r packs its tiles' pixels once
// its queued frames are on its film (rtg_film_gather: the handle's later folds wait for the pack, so
// the next frames' traversals run on meanwhile), sends them to devices[0] (one ncclSend / ncclRecv
// pair per rank inside one RCCL group), and devices[0] scatters every rank's pixels into the
// assembled film. No host wait.
int rtg_group_reduce_async(rtg_group* g) {
    if (!g) return RTG_ERR_ARG;
    if (g->poisoned) {
        g_err = "rtg_group_reduce: a rank failed its last render; the films are partial until rtg_group_clear";
        return RTG_ERR_ARG;
    }
    const size_t n = g->h.size();
    const size_t mp = std::max<uint32_t>(g->maxpix, 1);
    const uint32_t film_pixels = g->W * g->H;
    // timing: from rank 0's frames being on its film (a gather of no pixels is only that wait) to
    // the scatter's end; the other ranks' frames and the transfers are inside the pair
    if (int rc = rtg_film_gather(g->h[0], nullptr, 0, nullptr, g->xs[0])) return rc;
    HIPOK(hipSetDevice(g->devices[0]));
    HIPOK(hipEventRecord(g->xe0, g->xs[0]));
    if (n == 1 && !g->rccl_self) {
        // one device: its film is the film (one copy, not a pack and scatter of every pixel: C5's
        // 16.7M pixels took 0.97 ms that way); the handle's later folds wait for the copy
        HIPOK(hipMemcpyAsync(g->d_sum, g->h[0]->d_film, (size_t)film_pixels * 3 * sizeof(float), hipMemcpyDeviceToDevice,
                             g->xs[0]));
        HIPOK(hipEventRecord(g->xcopied, g->xs[0]));
        HIPOK(hipStreamWaitEvent(g->h[0]->stream, g->xcopied, 0));
        HIPOK(hipEventRecord(g->xe1, g->xs[0]));
        g->xtimed = true;
        g->reduced_spp = g->h[0]->spp;
        g->reduced = true;
        return RTG_OK;
    }
    // every rank packs its own tiles' pixels on its device (rank 0 straight into the receive buffer)
    for (size_t r = 0; r < n; ++r)
        if (int rc = rtg_film_gather(g->h[r], g->d_pix[r], g->npix[r], g->d_pack[r], g->xs[r])) return rc;
    if (!g->comms.empty()) {
        // one ncclSend per rank > 0 to device 0, which posts the matching ncclRecv into slot r of its
        // receive buffer. Every failure inside the group still closes it (ncclGroupEnd), so the
        // thread's RCCL group state stays balanced.
        if (g_rccl.group_start() != ncclSuccess) { g_err = "ncclGroupStart failed"; return RTG_ERR_HIP; }
        std::string fail;
        for (size_t r = g->rccl_self ? 0 : 1; r < n && fail.empty(); ++r) {
            if (!g->npix[r]) continue;
            const size_t cnt = (size_t)g->npix[r] * 3;
            ncclResult_t nr = g_rccl.send(g->d_pack[r], cnt, ncclFloat, 0, g->comms[r], g->xs[r]);
            if (nr == ncclSuccess)
                nr = g_rccl.recv(g->d_recv + r * mp * 3, cnt, ncclFloat, (int)r, g->comms[0], g->xs[0]);
            if (nr != ncclSuccess) fail = std::string("ncclSend/ncclRecv: ") + g_rccl.error_string(nr);
        }
        const ncclResult_t nr = g_rccl.group_end();
        if (!fail.empty()) { g_err = fail; return RTG_ERR_HIP; }
        if (nr != ncclSuccess) { g_err = std::string("ncclGroupEnd: ") + g_rccl.error_string(nr); return RTG_ERR_HIP; }
    } else if (n > 1) {
        // repeated devices: the packs move with device copies on devices[0]'s exchange stream, each
        // after its pack; the next packs wait for the copies
        for (size_t r = 1; r < n; ++r) {
            if (!g->npix[r]) continue;
            HIPOK(hipSetDevice(g->devices[r]));
            HIPOK(hipEventRecord(g->xpacked[r], g->xs[r]));
            HIPOK(hipSetDevice(g->devices[0]));
            HIPOK(hipStreamWaitEvent(g->xs[0], g->xpacked[r], 0));
            HIPOK(hipMemcpyPeerAsync(g->d_recv + r * mp * 3, g->devices[0], g->d_pack[r], g->devices[r],
                                     (size_t)g->npix[r] * 3 * sizeof(float), g->xs[0]));
        }
        HIPOK(hipSetDevice(g->devices[0]));
        HIPOK(hipEventRecord(g->xcopied, g->xs[0]));
        for (size_t r = 1; r < n; ++r) {
            HIPOK(hipSetDevice(g->devices[r]));
            HIPOK(hipStreamWaitEvent(g->xs[r], g->xcopied, 0));
        }
    }
    // tile supports cover the film, so the scatter writes every pixel of d_sum
    if (int rc = rtg_film_scatter(g->devices[0], g->d_recv, g->d_pix_all, (uint32_t)(n * mp), g->d_sum, film_pixels,
                                  g->xs[0]))
        return rc;
    HIPOK(hipEventRecord(g->xe1, g->xs[0]));
    g->xtimed = true;
    g->reduced_spp = g->h[0]->spp;
    g->reduced = true;
    return RTG_OK;
}

int rtg_group_reduce(rtg_group* g) {
    if (int rc = rtg_group_reduce_async(g)) return rc;
    return group_sync(g);
}

int rtg_group_synchronize(rtg_group* g) {
    if (!g) return RTG_ERR_ARG;
    return group_sync(g);
}

int rtg_group_film_read(rtg_group* g, float* rgb_sum, uint32_t* spp) {
    if (!g) return RTG_ERR_ARG;
    if (!g->reduced) {
        const int rc = rtg_group_reduce(g);
        if (rc) return rc;
    }
    HIPOK(hipSetDevice(g->devices[0]));
    HIPOK(hipStreamSynchronize(g->xs[0]));  // a queued exchange (the copy below does not order with it)
    if (rgb_sum) HIPOK(hipMemcpy(rgb_sum, g->d_sum, (size_t)g->W * g->H * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (spp) *spp = g->reduced_spp;
    return RTG_OK;
}

int rtg_group_clear(rtg_group* g) {
    if (!g) return RTG_ERR_ARG;
    if (int rc = group_sync(g)) return rc;
    for (rtg_handle* h : g->h) {
        const int rc = rtg_clear(h);
        if (rc) return rc;
    }
    g->reduced = false;
    g->poisoned = false;
    return RTG_OK;
}

double rtg_group_reduce_ms(rtg_group* g) { return g ? g->reduce_ms : 0.0; }

int rtg_group_uses_rccl(rtg_group* g) { return g && !g->comms.empty() ? 1 : 0; }

}  // extern "C"
