// Microbenchmark: what limits random per-lane gathers on gfx950 (instructions, lines or bytes)?
// Each lane walks a dependent random chain over a table of 64-B records, loading per step either
//   V=0: 4 x dwordx4 (64 B), V=1: 16 x dword (64 B), V=2: 1 x dwordx4 (16 B), V=3: 2 x dwordx4 (32 B),
//   V=4: 4 x dwordx4 with only 16 of 64 lanes active.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ inline unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int V>
__global__ __launch_bounds__(256) void k(const float4* __restrict__ tab, unsigned nrec, int steps, float* out) {
    const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (V == 4 && (threadIdx.x & 63) >= 16) return;
    unsigned idx = hash(gid) % nrec;
    float acc = 0.f;
    for (int s = 0; s < steps; ++s) {
        float sum = 0.f;
        const float4* r = tab + (size_t)idx * 4;
        if (V == 0 || V == 4) {
            float4 a = r[0], b = r[1], c = r[2], d = r[3];
            sum = a.x + b.y + c.z + d.w + a.w + b.x + c.y + d.z;
        } else if (V == 1) {
            const float* f = (const float*)r;
            float t[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) t[q] = __builtin_nontemporal_load(f + q) ;
#pragma unroll
            for (int q = 0; q < 16; ++q) sum += t[q];
        } else if (V == 2) {
            float4 a = r[0];
            sum = a.x + a.y + a.z + a.w;
        } else {
            float4 a = r[0], b = r[1];
            sum = a.x + b.y + a.z + b.w;
        }
        acc += sum;
        idx = hash(idx ^ __float_as_uint(sum)) % nrec;
    }
    out[gid] = acc;
}

template <int V>
void run(const float4* d, unsigned nrec, float* out, int blocks, int steps, const char* what) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        k<V><<<blocks, 256>>>(d, nrec, steps, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    const double lanes = (double)blocks * 256 * (V == 4 ? 0.25 : 1.0) * steps;
    printf("%-34s table %6.1f MiB blocks %5d: %7.2f G lane-steps/s\n", what, nrec * 64.0 / 1048576, blocks, lanes / ms / 1e6);
}

int main() {
    const size_t nf4 = (size_t)1 << 22;  // 64 MiB
    std::vector<float> h(nf4 * 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(i % 97) * 0.01f;
    float4* d; float* out;
    (void)hipMalloc(&d, h.size() * 4);
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 256 * 16 * 256 * 4);
    const int steps = 256;
    for (unsigned mb : {2u, 64u}) {
        const unsigned nrec = mb * 16384;
        for (int bl : {256 * 6, 256 * 12}) {
            run<0>(d, nrec, out, bl, steps, "64B as 4 x dwordx4");
            run<1>(d, nrec, out, bl, steps, "64B as 16 x dword");
            run<3>(d, nrec, out, bl, steps, "32B as 2 x dwordx4");
            run<2>(d, nrec, out, bl, steps, "16B as 1 x dwordx4");
            run<4>(d, nrec, out, bl, steps, "64B 4 x dwordx4, 16/64 lanes");
        }
    }
    return 0;
}
