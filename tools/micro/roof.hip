// roof.hip — the request-rate ceiling that bounds k_trace, and the FETCH_SIZE
// calibration for its access shape.
//
// k_trace is bound by vector-memory requests, not bytes: every lane of a node step issues four
// 16-B loads (global_load_dwordx4) of its own 64-B record at a data-dependent address, and the
// next record's address depends on this one. This kernel does exactly that and nothing else: per
// lane a dependent random chain of 64-B records (4 x dwordx4 each) over a table of T MiB, with V
// dependent VALU ops per step, at k_trace's occupancy (256-thread blocks, 6 waves per SIMD, 1536
// blocks on 256 CUs). It reports G 16-B requests/s = lanes x steps x 4 / time.
//
//   roof                      sweep: tables 1 / 21 / 69 / 1024 MiB x VALU 0 / 32 / 64 -> JSON lines
//   roof T V STEPS            one configuration (for rocprofv3 --pmc passes: FETCH_SIZE
//                             calibration on a table larger than the 256 MiB Infinity Cache)
// Build: hipcc --offload-arch=gfx950 -O3 -o roof roof.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

__device__ inline unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int VALU, int LOADS = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6)))
void k_chain(const float4* __restrict__ tab, unsigned nrec, int steps, float* out) {
    const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned idx = hash(gid * 2654435761u + 12345u) % nrec;
    float acc = 0.f;
    for (int s = 0; s < steps; ++s) {
        const float4* r = tab + (size_t)idx * LOADS;
        float4 v[LOADS];
#pragma unroll
        for (int k = 0; k < LOADS; ++k) v[k] = r[k];
        const float4 a = v[0];
        float sum = 0.0f;
#pragma unroll
        for (int k = 0; k < LOADS; ++k) sum += (v[k].x + v[k].y) + (v[k].z + v[k].w);
#pragma unroll
        for (int v = 0; v < VALU; ++v) sum = __builtin_fmaf(sum, 1.0000001f, a.y * (float)v);
        acc += sum;
        idx = hash(idx ^ __float_as_uint(sum)) % nrec;
    }
    out[gid] = acc;
}

template <int LOADS, int VALU = 64>
static double run_l(const float4* d, unsigned nrec, float* out, int blocks, int steps, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < reps; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((k_chain<VALU, LOADS>), dim3(blocks), dim3(256), 0, 0, d, nrec, steps, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

static double run(int valu, const float4* d, unsigned nrec, float* out, int blocks, int steps, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < reps; ++rep) {
        (void)hipEventRecord(a);
        switch (valu) {
            case 0: hipLaunchKernelGGL(k_chain<0>, dim3(blocks), dim3(256), 0, 0, d, nrec, steps, out); break;
            case 32: hipLaunchKernelGGL(k_chain<32>, dim3(blocks), dim3(256), 0, 0, d, nrec, steps, out); break;
            default: hipLaunchKernelGGL(k_chain<64>, dim3(blocks), dim3(256), 0, 0, d, nrec, steps, out); break;
        }
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return best;
}

int main(int argc, char** argv) {
    int dev_cus = 0;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = (dev_cus > 0 ? dev_cus : 256) * 6;  // 6 waves per SIMD, 4 SIMDs, 4 waves per block
    const size_t maxmib = 1024;
    const size_t nfl = maxmib * 1048576 / 4;
    float4* d = nullptr;
    float* out = nullptr;
    if (hipMalloc(&d, nfl * 4) != hipSuccess || hipMalloc(&out, (size_t)(dev_cus > 0 ? dev_cus : 256) * 16 * 256 * 4) != hipSuccess) {
        std::fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    {
        std::vector<float> h(nfl);
        for (size_t i = 0; i < nfl; ++i) h[i] = (float)(i % 97) * 0.01f;
        (void)hipMemcpy(d, h.data(), nfl * 4, hipMemcpyHostToDevice);
    }
    auto one = [&](size_t mib, int valu, int steps, int reps) {
        const unsigned nrec = (unsigned)(mib * 1048576 / 64);
        const double ms = run(valu, d, nrec, out, blocks, steps, reps);
        const double lanes = (double)blocks * 256;
        const double req = lanes * steps * 4;
        std::printf("{\"table_mib\": %zu, \"valu_per_step\": %d, \"blocks\": %d, \"steps\": %d, \"ms\": %.4f, "
                    "\"g_req_per_s\": %.2f, \"g_lane_steps_per_s\": %.2f, \"record_bytes\": %.0f, "
                    "\"requested_gbs\": %.1f}\n",
                    mib, valu, blocks, steps, ms, req / ms / 1e6, lanes * steps / ms / 1e6, lanes * steps * 64.0,
                    lanes * steps * 64.0 / ms / 1e6);
        std::fflush(stdout);
    };
    if (argc == 2 && std::string(argv[1]) == "width") {
        // records of 1-8 dwordx4 loads, equal bytes per lane: the same 69 MiB table, 64 VALU per step
        const size_t mib = 69;
        for (int loads : {1, 2, 3, 4, 6, 8}) {
            const unsigned nrec = (unsigned)(mib * 1048576 / (16 * loads));
            const int steps = 1024 / loads;  // equal bytes per lane
            const double ms = loads == 1 ? run_l<1>(d, nrec, out, blocks, steps, 3)
                            : loads == 2 ? run_l<2>(d, nrec, out, blocks, steps, 3)
                            : loads == 3 ? run_l<3>(d, nrec, out, blocks, steps, 3)
                            : loads == 4 ? run_l<4>(d, nrec, out, blocks, steps, 3)
                            : loads == 6 ? run_l<6>(d, nrec, out, blocks, steps, 3)
                                         : run_l<8>(d, nrec, out, blocks, steps, 3);
            std::printf("{\"record_loads\": %d, \"valu_per_step\": 64, \"steps\": %d, \"ms\": %.4f, \"g_req_per_s\": %.1f, \"g_steps_per_s\": %.1f}\n",
                        loads, steps, ms, (double)blocks * 256 * steps * loads / ms / 1e6,
                        (double)blocks * 256 * steps / ms / 1e6);
        }
        for (int loads : {1, 2, 4}) {  // the same without VALU between the steps
            const unsigned nrec = (unsigned)(mib * 1048576 / (16 * loads));
            const int steps = 1024 / loads;
            const double ms = loads == 1 ? run_l<1, 0>(d, nrec, out, blocks, steps, 3)
                            : loads == 2 ? run_l<2, 0>(d, nrec, out, blocks, steps, 3)
                                         : run_l<4, 0>(d, nrec, out, blocks, steps, 3);
            std::printf("{\"record_loads\": %d, \"valu_per_step\": 0, \"steps\": %d, \"ms\": %.4f, \"g_req_per_s\": %.1f, \"g_steps_per_s\": %.1f}\n",
                        loads, steps, ms, (double)blocks * 256 * steps * loads / ms / 1e6,
                        (double)blocks * 256 * steps / ms / 1e6);
        }
        return 0;
    }
    if (argc == 2 && std::string(argv[1]) == "occ") {
        // chains in flight: blocks per CU = waves per SIMD (4 waves per block), 64-B records, 69 MiB
        const size_t mib = 69;
        const unsigned nrec = (unsigned)(mib * 1048576 / 64);
        const int cus = dev_cus > 0 ? dev_cus : 256;
        for (int wps : {1, 2, 3, 4, 6, 8, 12, 16}) {
            const int nb = cus * wps;
            const int steps = 256;
            const double ms = run_l<4>(d, nrec, out, nb, steps, 3);
            std::printf("{\"waves_per_simd\": %d, \"blocks\": %d, \"ms\": %.4f, \"g_steps_per_s\": %.1f}\n", wps, nb,
                        ms, (double)nb * 256 * steps / ms / 1e6);
        }
        return 0;
    }
    if (argc >= 4) {
        one((size_t)std::atoi(argv[1]), std::atoi(argv[2]), std::atoi(argv[3]), 1);
    } else {
        for (size_t mib : {1, 21, 69, 1024})
            for (int valu : {0, 32, 64}) one(mib, valu, 256, 3);
    }
    (void)hipFree(d);
    (void)hipFree(out);
    return 0;
}
