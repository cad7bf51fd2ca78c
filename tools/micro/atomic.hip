// Microbenchmark: is k_shade's block-level compaction (one device-scope atomicAdd per 256-path block
// on each of two queue counters) bound by the same-address atomic rate? A grid of G blocks of 256
// threads; each block reads 64 B per thread, writes 16 B per thread and, in V=1, thread 0 issues one
// returning atomicAdd on each of two counters (in separate 128-B lines), V=0 none, V=2 the atomics
// spread over 8 counter pairs (blockIdx % 8), V=3 one atomic per block on one counter only.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V>
__global__ __launch_bounds__(256) void k(const float4* __restrict__ in, float4* __restrict__ out, unsigned* ctr, unsigned n) {
    __shared__ unsigned base[2];
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.x * 256 >= n) return;
    float4 a = in[2 * i], b = in[2 * i + 1];
    float4 c = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    if (threadIdx.x == 0) {
        unsigned* p = ctr + (V == 2 ? (blockIdx.x & 7) * 64 : 0);
        base[0] = V ? atomicAdd(p, 200u) : 0u;
        base[1] = (V == 1 || V == 2) ? atomicAdd(p + 32, 150u) : 0u;
    }
    __syncthreads();
    c.x += (float)(base[0] & 1) + (float)(base[1] & 1);
    out[i] = c;
}

template <int V>
void run(const float4* in, float4* out, unsigned* ctr, unsigned n, const char* what) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const unsigned g = n / 256;
    hipLaunchKernelGGL(k<V>, dim3(g), dim3(256), 0, 0, in, out, ctr, n);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<V>, dim3(g), dim3(256), 0, 0, in, out, ctr, n);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    printf("{\"variant\": \"%s\", \"blocks\": %u, \"ms\": %.4f, \"blocks_per_us\": %.1f, \"atomics_per_s_per_counter\": %.3g}\n",
           what, g, ms, g / (ms * 1e3), (V == 0 ? 0.0 : V == 2 ? g / 8.0 : (double)g) / (ms * 1e-3));
}

int main() {
    const unsigned n = 64u << 20;  // 64M "paths", 262144 blocks (C3 bounce 0)
    float4 *in, *out;
    unsigned* ctr;
    (void)hipMalloc(&in, (size_t)n * 32);
    (void)hipMalloc(&out, (size_t)n * 16);
    (void)hipMalloc(&ctr, 64 * 8 * sizeof(unsigned));
    (void)hipMemset(in, 0, (size_t)n * 32);
    (void)hipMemset(ctr, 0, 64 * 8 * sizeof(unsigned));
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(in, out, ctr, n, "no atomics");
        run<3>(in, out, ctr, n, "1 atomic per block, 1 counter");
        run<1>(in, out, ctr, n, "2 atomics per block, 2 counters");
        run<2>(in, out, ctr, n, "2 atomics per block, 8 counter pairs");
    }
    return 0;
}
