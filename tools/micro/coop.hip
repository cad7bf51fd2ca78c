// Microbenchmark: is a per-lane random 64-B record fetch cheaper when 4 lanes fetch one record
// together (one 64-B piece per wave-instruction per lane quad) and the records are redistributed
// through LDS? Models one traversal node step: dependent random chain, VALU work per step.
//   A: per lane 4 x global_load_dwordx4 of its own record (what k_trace does today)
//   B: cooperative: instruction k, lane L loads piece L&3 of the record of lane (L&~3)+k (owner index
//      by DPP quad broadcast), ds_write_b128 into [owner][piece], then each lane ds_read_b128 x4
//   C: cooperative via global_load_lds_dwordx4 (LDS-DMA, lane-linear image), then ds_read_b128 x4
// Build: hipcc --offload-arch=gfx950 -O3 -o coop coop.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ inline unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int K>
__device__ inline unsigned quad_bcast(unsigned v) {
    // quad_perm [K,K,K,K]
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, K | (K << 2) | (K << 4) | (K << 6), 0xf, 0xf, false);
}

template <int MODE, int VALU>
__global__ __launch_bounds__(256) void k(const float4* __restrict__ tab, unsigned nrec, int steps, float* out,
                                         unsigned active) {
    __shared__ float4 st[4][4][64];  // [wave][piece-instruction k][lane] : 4 KB per wave
    const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned idx = hash(gid) % nrec;
    float acc = 0.f;
    const bool on = (unsigned)lane < active;
    for (int s = 0; s < steps; ++s) {
        float4 a, b, c, d;
        if (MODE == 0) {
            if (on) {
                const float4* r = tab + (size_t)idx * 4;
                a = r[0]; b = r[1]; c = r[2]; d = r[3];
            } else {
                a = b = c = d = make_float4(0, 0, 0, 0);
            }
        } else {
            const unsigned i0 = quad_bcast<0>(idx), i1 = quad_bcast<1>(idx), i2 = quad_bcast<2>(idx),
                           i3 = quad_bcast<3>(idx);
            const int pc = lane & 3;
            if (MODE == 1) {
                const float4 l0 = tab[(size_t)i0 * 4 + pc];
                const float4 l1 = tab[(size_t)i1 * 4 + pc];
                const float4 l2 = tab[(size_t)i2 * 4 + pc];
                const float4 l3 = tab[(size_t)i3 * 4 + pc];
                st[wave][0][lane] = l0;
                st[wave][1][lane] = l1;
                st[wave][2][lane] = l2;
                st[wave][3][lane] = l3;
            } else {
                __builtin_amdgcn_global_load_lds(tab + (size_t)i0 * 4 + pc, &st[wave][0][0], 16, 0, 0);
                __builtin_amdgcn_global_load_lds(tab + (size_t)i1 * 4 + pc, &st[wave][1][0], 16, 0, 0);
                __builtin_amdgcn_global_load_lds(tab + (size_t)i2 * 4 + pc, &st[wave][2][0], 16, 0, 0);
                __builtin_amdgcn_global_load_lds(tab + (size_t)i3 * 4 + pc, &st[wave][3][0], 16, 0, 0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // record of lane L = st[wave][L&3][(L&~3) + 0..3]
            const float4* mine = &st[wave][pc][lane & ~3];
            a = mine[0]; b = mine[1]; c = mine[2]; d = mine[3];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        float sum = (((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w))) + (((c.x + c.y) + (c.z + c.w)) + ((d.x + d.y) + (d.z + d.w)));
#pragma unroll
        for (int v = 0; v < VALU; ++v) sum = __builtin_fmaf(sum, 1.0000001f, a.y * (float)v);
        acc += sum;
        idx = hash(idx ^ __float_as_uint(sum)) % nrec;
    }
    out[gid] = acc;
}

template <int MODE, int VALU>
double run(const float4* d, unsigned nrec, float* out, int blocks, int steps, unsigned active) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        k<MODE, VALU><<<blocks, 256>>>(d, nrec, steps, out, active);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    return (double)blocks * 4 * active * steps / ms / 1e6;  // G lane-steps/s
}

int main() {
    const size_t maxrec = (size_t)1 << 22;  // 4M records x 64 B = 256 MiB
    std::vector<float> h(maxrec * 16);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(i % 97) * 0.01f;
    float4* d; float* out;
    (void)hipMalloc(&d, h.size() * 4);
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 256 * 8 * 256 * 4);
    const int steps = 512;
    const int blocks = 256 * 6;
    for (size_t mb : {2, 21, 85}) {
        const unsigned nrec = (unsigned)(mb * 1048576 / 64);
        printf("table %3zu MiB  VALU 0  : A %6.2f  B %6.2f  C %6.2f  G lane-steps/s\n", mb,
               run<0, 0>(d, nrec, out, blocks, steps, 64), run<1, 0>(d, nrec, out, blocks, steps, 64),
               run<2, 0>(d, nrec, out, blocks, steps, 64));
        printf("table %3zu MiB  VALU 64 : A %6.2f  B %6.2f  C %6.2f\n", mb,
               run<0, 64>(d, nrec, out, blocks, steps, 64), run<1, 64>(d, nrec, out, blocks, steps, 64),
               run<2, 64>(d, nrec, out, blocks, steps, 64));
        printf("table %3zu MiB  VALU 128: A %6.2f  B %6.2f  C %6.2f\n", mb,
               run<0, 128>(d, nrec, out, blocks, steps, 64), run<1, 128>(d, nrec, out, blocks, steps, 64),
               run<2, 128>(d, nrec, out, blocks, steps, 64));
    }
    // 40 of 64 lanes active (traversal lane utilisation ~0.65): does A get cheaper per step?
    const unsigned nrec = 21u * 1048576 / 64;
    printf("21 MiB, 40/64 lanes, VALU 64: A %6.2f (per active lane)\n", run<0, 64>(d, nrec, out, blocks, steps, 40));
    for (int bl : {256 * 4, 256 * 8}) {
        printf("21 MiB, blocks %d, VALU 64: A %6.2f  B %6.2f  C %6.2f\n", bl, run<0, 64>(d, nrec, out, bl, steps, 64),
               run<1, 64>(d, nrec, out, bl, steps, 64), run<2, 64>(d, nrec, out, bl, steps, 64));
    }
    return 0;
}
