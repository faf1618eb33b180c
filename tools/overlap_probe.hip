// SUPERSEDED by tools/cost_probe.hip (round 2).  The specialised case below
// picks roles by (threadIdx.x >> 6) & 1, which puts every lookup wave on two
// SIMDs (waves go to SIMDs in the cyclic order 0,2,1,3): it measures SIMD
// placement, not LDS/VALU overlap, and its "the times add" conclusion was
// withdrawn.  Kept for the record of round 1.
// overlap_probe.hip — do LDS lookups and VALU work overlap on gfx950?
//
// Three kernels with the same launch shape as the token kernels (1024
// threads, 128 KiB LDS, one workgroup per CU): LDS-only (ds_read_b32 lookups
// with the replicated-table address pattern), VALU-only (full-rate v_bitop3
// chains), and both interleaved.  If t(both) ~ max(t_lds, t_valu) they
// overlap; if ~ sum they compete for a shared resource.
//   hipcc --offload-arch=gfx950 -O3 -o build_tools/overlap_probe tools/overlap_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef __attribute__((address_space(3))) const uint32_t l32;

template <int LDS_PER_ITER, int VALU_PER_ITER, bool PERM>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t seed, int iters) {
    extern __shared__ uint32_t tab[];
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) tab[i] = i * 2654435761u + seed;
    __syncthreads();
    const uint32_t lane = 4u * (threadIdx.x & 31u);
    uint32_t x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = (threadIdx.x * 977u + j * 131u) & 0xff00u;
    uint32_t v0 = threadIdx.x ^ seed, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11, v5 = v0 * 13, v6 = v0 * 17, v7 = v0 * 19;
    uint32_t c1 = seed * 7 + 1 + threadIdx.x, c2 = seed * 11 + 3;
    uint32_t mask = 0xff00u;
    asm volatile("" : "+v"(c1), "+v"(c2), "+v"(mask));   // VGPR operands (SGPR operands halve VALU rate)
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < LDS_PER_ITER; ++j) {
            uint32_t a;
            if (PERM) a = __builtin_amdgcn_perm(x[j & 15], lane, 0x0C0C0500u);
            else a = __builtin_amdgcn_bitop3_b32(x[j & 15], mask, lane, 0xEA);
            x[j & 15] ^= *(l32 *)(uintptr_t)(a + ((j & 1) ? 128 : 0));
        }
#pragma unroll
        for (int j = 0; j < VALU_PER_ITER / 8; ++j) {
            v0 = __builtin_amdgcn_bitop3_b32(v0, c1, c2, 0x96); v1 = __builtin_amdgcn_bitop3_b32(v1, c1, c2, 0x96);
            v2 = __builtin_amdgcn_bitop3_b32(v2, c1, c2, 0x96); v3 = __builtin_amdgcn_bitop3_b32(v3, c1, c2, 0x96);
            v4 = __builtin_amdgcn_bitop3_b32(v4, c1, c2, 0x96); v5 = __builtin_amdgcn_bitop3_b32(v5, c1, c2, 0x96);
            v6 = __builtin_amdgcn_bitop3_b32(v6, c1, c2, 0x96); v7 = __builtin_amdgcn_bitop3_b32(v7, c1, c2, 0x96);
        }
    }
    uint32_t acc = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int L, int V, bool P>
static int run(const char *name, uint32_t *out, int ncu, int iters) {
    auto kern = k<L, V, P>;
    CHECK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(1024), 131072, 0, out, 1u, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kern, dim3(ncu), dim3(1024), 131072, 0, out, 2u + r, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double waves_per_simd = 4.0;
    const double lds_instr_per_cu = 16.0 * L * iters;           // wave-instructions per CU
    const double valu_instr_per_simd = waves_per_simd * (V + (P ? L : 2.0 * L) + L) * iters;
    printf("%-34s %8.3f ms   LDS %.2f cyc/ds_read/CU   VALU %.2f cyc/instr/SIMD (at 2.4 GHz)\n", name, best,
           best * 1e-3 * 2.4e9 / (lds_instr_per_cu ? lds_instr_per_cu : 1),
           best * 1e-3 * 2.4e9 / valu_instr_per_simd);
    return 0;
}


// Same total work as k<L, V, false>, but specialised by wave: even waves do
// the lookups of two waves, odd waves the VALU of two waves.
template <int LDS_PER_ITER, int VALU_PER_ITER>
__global__ __launch_bounds__(1024) void k_spec(uint32_t *out, uint32_t seed, int iters) {
    extern __shared__ uint32_t tab[];
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) tab[i] = i * 2654435761u + seed;
    __syncthreads();
    const uint32_t lane = 4u * (threadIdx.x & 31u);
    const bool lds_wave = ((threadIdx.x >> 6) & 1u) == 0;
    uint32_t x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = (threadIdx.x * 977u + j * 131u) & 0xff00u;
    uint32_t v0 = threadIdx.x ^ seed, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11, v5 = v0 * 13, v6 = v0 * 17, v7 = v0 * 19;
    uint32_t c1 = seed * 7 + 1 + threadIdx.x, c2 = seed * 11 + 3;
    uint32_t mask = 0xff00u;
    asm volatile("" : "+v"(c1), "+v"(c2), "+v"(mask));
    if (lds_wave) {
        for (int it = 0; it < 2 * iters; ++it) {
#pragma unroll
            for (int j = 0; j < LDS_PER_ITER; ++j) {
                const uint32_t a = __builtin_amdgcn_bitop3_b32(x[j & 15], mask, lane, 0xEA);
                x[j & 15] ^= *(l32 *)(uintptr_t)(a + ((j & 1) ? 128 : 0));
            }
        }
    } else {
        for (int it = 0; it < 2 * iters; ++it) {
#pragma unroll
            for (int j = 0; j < VALU_PER_ITER / 8; ++j) {
                v0 = __builtin_amdgcn_bitop3_b32(v0, c1, c2, 0x96); v1 = __builtin_amdgcn_bitop3_b32(v1, c1, c2, 0x96);
                v2 = __builtin_amdgcn_bitop3_b32(v2, c1, c2, 0x96); v3 = __builtin_amdgcn_bitop3_b32(v3, c1, c2, 0x96);
                v4 = __builtin_amdgcn_bitop3_b32(v4, c1, c2, 0x96); v5 = __builtin_amdgcn_bitop3_b32(v5, c1, c2, 0x96);
                v6 = __builtin_amdgcn_bitop3_b32(v6, c1, c2, 0x96); v7 = __builtin_amdgcn_bitop3_b32(v7, c1, c2, 0x96);
            }
        }
    }
    uint32_t acc = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int L, int V>
static int run_spec(const char *name, uint32_t *out, int ncu, int iters) {
    auto kern = k_spec<L, V>;
    CHECK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(1024), 131072, 0, out, 1u, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kern, dim3(ncu), dim3(1024), 131072, 0, out, 2u + r, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    printf("%-34s %8.3f ms   (wave-specialised: even waves LDS x2, odd waves VALU x2)\n", name, best);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount, iters = 20000;
    uint32_t *out;
    CHECK(hipMalloc(&out, 4ull * ncu * 1024));
    run<16, 0, false>("lds16 (and_or addr)", out, ncu, iters);
    run<16, 16, false>("lds16 + valu16", out, ncu, iters);
    run<0, 64, false>("valu64 bitop3", out, ncu, iters);
    run<16, 64, false>("lds16 + valu64", out, ncu, iters);
    run<0, 32, false>("valu32 bitop3", out, ncu, iters);
    run<16, 32, false>("lds16 + valu32", out, ncu, iters);
    run<16, 0, true>("lds16 (perm addr)", out, ncu, iters);
    run<16, 64, true>("lds16 (perm) + valu64", out, ncu, iters);
    run<16, 128, false>("lds16 + valu128", out, ncu, iters);
    run_spec<16, 64>("spec lds16 | valu64", out, ncu, iters);
    run_spec<16, 128>("spec lds16 | valu128", out, ncu, iters);
    run<0, 128, false>("valu128 bitop3", out, ncu, iters);
    return 0;
}
