// Microbenchmark: per-lane random 128-B node fetch (8 x dwordx4, 64 distinct lines per
// wave-instruction) vs cooperative fetch (8 lanes share one node: 8 lines per wave-instruction)
// followed by an in-register 8x8 transpose (ds_bpermute). Dependent chains model traversal.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ inline unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int MODE, int NF>
__global__ __launch_bounds__(256) void k(const float4* __restrict__ tab, unsigned nnodes, int steps, float* out) {
    const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned idx = hash(gid) % nnodes;
    float acc = 0.f;
    const int lane = threadIdx.x & 63;
    for (int s = 0; s < steps; ++s) {
        float4 v[8] = {};
        if (MODE == 0) {
#pragma unroll
            for (int q = 0; q < NF; ++q) v[q] = tab[(size_t)idx * NF + q];
        } else {
            const int g = lane & ~7, j = lane & 7;
            float4 c[8];
#pragma unroll
            for (int k2 = 0; k2 < 8; ++k2) {
                const unsigned other = __shfl(idx, g + k2);
                c[k2] = tab[(size_t)other * NF + j];
            }
            // lane g+L needs chunk q of node N_{g+L}: lane g+q holds it in c[L].
            // round r: receiver L reads lane g+((L+r)&7), which sends c[(j-r)&7].
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int ks = (j - r) & 7;
                float4 send = c[0];
#pragma unroll
                for (int k2 = 1; k2 < 8; ++k2) if (ks == k2) send = c[k2];
                const int src = g + ((j + r) & 7);
                float4 got;
                got.x = __shfl(send.x, src);
                got.y = __shfl(send.y, src);
                got.z = __shfl(send.z, src);
                got.w = __shfl(send.w, src);
                const int qd = (j + r) & 7;  // chunk index received
#pragma unroll
                for (int k2 = 0; k2 < 8; ++k2) if (qd == k2) v[k2] = got;
            }
        }
        float sum = 0.f;
#pragma unroll
        for (int q = 0; q < NF; ++q) sum += v[q].x + v[q].y + v[q].z + v[q].w;
        acc += sum;
        idx = hash(idx ^ __float_as_uint(sum)) % nnodes;
    }
    out[gid] = acc;
}

template <int NF>
void run(const float4* d, unsigned nnodes, float* out, int blocks, int steps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        k<0, NF><<<blocks, 256>>>(d, nnodes, steps, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        double fetches = (double)blocks * 256 * steps;
        if (rep == 2) printf("node %3d B, table %6.1f MiB, blocks %d: %.2f G fetches/s  %.2f TB/s\n", NF * 16,
                             nnodes * NF * 16.0 / 1048576, blocks, fetches / ms / 1e6, fetches * NF * 16 / ms / 1e9);
    }
}

int main() {
    const size_t maxf = (size_t)1 << 24;  // 256 MiB of float4... (4M float4 = 64 MiB)
    std::vector<float> h(maxf * 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(i % 97) * 0.01f;
    float4* d; float* out;
    hipMalloc(&d, h.size() * 4);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&out, 256 * 8 * 256 * 4);
    const int steps = 256;
    for (size_t mb : {4, 16, 64, 256}) {
        const size_t f4 = mb * 65536;
        run<8>(d, f4 / 8, out, 256 * 6, steps);
        run<4>(d, f4 / 4, out, 256 * 6, steps);
        run<2>(d, f4 / 2, out, 256 * 6, steps);
    }
    run<4>(d, (64 * 65536) / 4, out, 256 * 8, steps);
    run<4>(d, (64 * 65536) / 4, out, 256 * 4, steps);
    return 0;
}
