// rtg_multi.hip — one-node multi-GPU rendering behind the C-ABI (include/rtg.h, rtg_group_*).
//
// RTBase's only parallelism is the tile pool of RayTracer::pathTracerTileBased (Renderer.h:836-853:
// numProcs threads pop 32x32 tiles from a shared queue, Renderer.h:52-54). Here the tiles are
// spread over the GPUs of one node instead: device r renders every sample of the tiles with
// (tile_x + tile_y) % N == r (diagonal stripes, the same partition as raytracingrenderer_amd/
// distributed.py), one host thread and one rtg_handle per device, and the float films are summed
// into the first device with one RCCL reduce over xGMI (ncclCommInitAll over the devices, single
// process). Tile supports are disjoint and every other device adds +0.0, so the reduced film is
// bit-identical to a one-GPU render, whatever the reduction order.
//
// A device list that repeats a device (rehearsing N ranks on one GPU) cannot form an RCCL
// communicator; the ranks then render one after another, each with an equal share of the device's
// memory for its chunks (rtg_handle::mem_cap), and the films are summed through host memory in
// rank order (same bits).
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
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {
struct Rccl {
    bool tried = false, ok = false;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t, hipStream_t) = nullptr;
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
    g_rccl.reduce = (decltype(g_rccl.reduce))dlsym(h, "ncclReduce");
    g_rccl.group_start = (decltype(g_rccl.group_start))dlsym(h, "ncclGroupStart");
    g_rccl.group_end = (decltype(g_rccl.group_end))dlsym(h, "ncclGroupEnd");
    g_rccl.error_string = (decltype(g_rccl.error_string))dlsym(h, "ncclGetErrorString");
    g_rccl.ok = g_rccl.comm_init_all && g_rccl.comm_destroy && g_rccl.reduce && g_rccl.group_start &&
                g_rccl.group_end && g_rccl.error_string;
    if (!g_rccl.ok) g_err = "RCCL: missing symbols";
    return g_rccl.ok;
}

// the reduce's two timing events on device 0, destroyed on every return path
struct EventPair {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    ~EventPair() {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    }
};
}  // namespace

struct rtg_group {
    std::vector<int> devices;
    std::vector<rtg_handle*> h;
    std::vector<std::vector<uint32_t>> tiles;  // per rank
    std::vector<ncclComm_t> comms;             // empty: host reduce (repeated devices)
    float* d_sum = nullptr;                    // reduced film on devices[0]
    uint32_t W = 0, H = 0;
    uint32_t reduced_spp = 0;
    bool reduced = false;
    bool distinct = true;                      // every rank on its own device (RCCL, concurrent ranks)
    bool poisoned = false;                     // a rank failed a render: films hold partial samples
    double reduce_ms = 0.0;
    double prepare_ms = 0.0, upload_ms = 0.0;  // group setup: host build once, parallel uploads
};

extern "C" {

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
    for (ncclComm_t c : g->comms) (void)g_rccl.comm_destroy(c);
    if (g->d_sum) {
        (void)hipSetDevice(g->devices[0]);
        (void)hipFree(g->d_sum);
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
    if (g->distinct) {
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
    if (hipSetDevice(g->devices[0]) != hipSuccess ||
        hipMalloc((void**)&g->d_sum, (size_t)g->W * g->H * 3 * sizeof(float)) != hipSuccess) {
        g_err = "rtg_group_create: film allocation failed";
        rtg_group_destroy(g);
        return RTG_ERR_HIP;
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
    const size_t n = g->h.size();
    std::vector<int> rc(n, RTG_OK);
    std::vector<std::string> err(n);
    auto run = [&](size_t r) {
        const std::vector<uint32_t>& t = g->tiles[r];
        if (t.empty()) return;  // more devices than tiles: this rank's film stays zero
        rc[r] = rtg_render(g->h[r], first_sample, n_samples, seed, t.data(), (uint32_t)t.size());
        if (rc[r]) err[r] = rtg_last_error();  // g_err is thread-local
    };
    if (n == 1 || !g->distinct) {
        for (size_t r = 0; r < n; ++r) run(r);  // one device: ranks in turn
    } else {
        std::vector<std::thread> pool;
        for (size_t r = 0; r < n; ++r) pool.emplace_back(run, r);
        for (auto& t : pool) t.join();
    }
    g->reduced = false;
    for (size_t r = 0; r < n; ++r)
        if (rc[r]) {
            g->poisoned = true;
            g_err = "rank " + std::to_string(r) + ": " + err[r] + " (group films now partial: rtg_group_clear)";
            return rc[r];
        }
    return RTG_OK;
}

int rtg_group_reduce(rtg_group* g) {
    if (!g) return RTG_ERR_ARG;
    if (g->poisoned) {
        g_err = "rtg_group_reduce: a rank failed its last render; the films are partial until rtg_group_clear";
        return RTG_ERR_ARG;
    }
    const size_t n = g->h.size();
    const size_t count = (size_t)g->W * g->H * 3;
    EventPair ev;
    HIPOK(hipSetDevice(g->devices[0]));
    HIPOK(hipEventCreate(&ev.e0));
    HIPOK(hipEventCreate(&ev.e1));
    HIPOK(hipEventRecord(ev.e0, g->h[0]->stream));
    if (!g->comms.empty()) {
        // every rank's film (summed in sample order on its device) -> device 0, ncclSum. Every
        // failure inside the group still closes it (ncclGroupEnd), so the thread's RCCL group
        // state stays balanced.
        if (g_rccl.group_start() != ncclSuccess) { g_err = "ncclGroupStart failed"; return RTG_ERR_HIP; }
        std::string fail;
        for (size_t r = 0; r < n && fail.empty(); ++r) {
            const hipError_t he = hipSetDevice(g->devices[r]);
            if (he != hipSuccess) {
                fail = std::string("hipSetDevice: ") + hipGetErrorString(he);
                break;
            }
            const ncclResult_t nr = g_rccl.reduce(g->h[r]->d_film, r == 0 ? g->d_sum : nullptr, count, ncclFloat, ncclSum,
                                                  0, g->comms[r], g->h[r]->stream);
            if (nr != ncclSuccess) fail = std::string("ncclReduce: ") + g_rccl.error_string(nr);
        }
        const ncclResult_t nr = g_rccl.group_end();
        if (!fail.empty()) { g_err = fail; return RTG_ERR_HIP; }
        if (nr != ncclSuccess) { g_err = std::string("ncclGroupEnd: ") + g_rccl.error_string(nr); return RTG_ERR_HIP; }
        for (size_t r = 0; r < n; ++r) {
            HIPOK(hipSetDevice(g->devices[r]));
            HIPOK(hipStreamSynchronize(g->h[r]->stream));
        }
    } else {
        // repeated devices: rank order through host memory
        std::vector<float> sum(count, 0.0f), f(count);
        for (size_t r = 0; r < n; ++r) {
            uint32_t spp = 0;
            const int rc = rtg_film_read(g->h[r], f.data(), &spp);
            if (rc) return rc;
            for (size_t i = 0; i < count; ++i) sum[i] = sum[i] + f[i];
        }
        HIPOK(hipSetDevice(g->devices[0]));
        HIPOK(hipMemcpy(g->d_sum, sum.data(), count * sizeof(float), hipMemcpyHostToDevice));
    }
    HIPOK(hipSetDevice(g->devices[0]));
    HIPOK(hipEventRecord(ev.e1, g->h[0]->stream));
    HIPOK(hipEventSynchronize(ev.e1));
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, ev.e0, ev.e1);
    g->reduce_ms = ms;
    g->reduced_spp = g->h[0]->spp;
    g->reduced = true;
    return RTG_OK;
}

int rtg_group_film_read(rtg_group* g, float* rgb_sum, uint32_t* spp) {
    if (!g) return RTG_ERR_ARG;
    if (!g->reduced) {
        const int rc = rtg_group_reduce(g);
        if (rc) return rc;
    }
    HIPOK(hipSetDevice(g->devices[0]));
    if (rgb_sum) HIPOK(hipMemcpy(rgb_sum, g->d_sum, (size_t)g->W * g->H * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (spp) *spp = g->reduced_spp;
    return RTG_OK;
}

int rtg_group_clear(rtg_group* g) {
    if (!g) return RTG_ERR_ARG;
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
