// issue_probe.hip — VALU issue rate per SIMD as a function of waves per SIMD
// and independent chains per wave (gfx950).  Each wave runs CH independent
// v_bitop3_b32 chains (VGPR operands only); LDS is allocated only to pin the
// number of workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 -o build_tools/issue_probe tools/issue_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#ifndef INSN
#define INSN "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96"
#endif
#ifndef BCON
#define BCON "v"
#endif
template <int CH>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t seed, int iters) {
    extern __shared__ uint32_t pin[];
    uint32_t v[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) v[j] = threadIdx.x * (j + 3) ^ seed;
    uint32_t b = BCON[0] == 's' ? seed * 7 : threadIdx.x * 7 + seed, c = threadIdx.x * 13 + 1;
    asm volatile("" : "+" BCON(b), "+v"(c));
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 64 / CH; ++r)
#pragma unroll
            for (int j = 0; j < CH; ++j) asm volatile(INSN : "+v"(v[j]) : BCON(b), "v"(c));
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) acc ^= v[j];
    if (acc == 0x12345678u) pin[0] = acc;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int CH>
static int run(int ncu, uint32_t *out, int threads, int wg_per_cu) {
    auto kern = k<CH>;
    const size_t lds = wg_per_cu == 1 ? 100 * 1024 : 40 * 1024;
    CHECK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int iters = 4000, blocks = ncu * wg_per_cu;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, 0, out, 1u, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, 0, out, 2u + r, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double waves_per_simd = threads / 64.0 * wg_per_cu / 4.0;
    const double instr_per_simd = waves_per_simd * 64.0 * iters;
    printf("chains/wave %2d  waves/SIMD %4.1f : %.3f ms  %.2f cyc/instr/SIMD @2.4GHz  (per wave: %.1f cyc/instr)\n", CH,
           waves_per_simd, best, best * 1e-3 * 2.4e9 / instr_per_simd,
           best * 1e-3 * 2.4e9 / instr_per_simd * waves_per_simd);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    uint32_t *out;
    CHECK(hipMalloc(&out, 4ull * ncu * 2048));
    printf("%s  [b operand: %s]\n", INSN, BCON);
    run<8>(ncu, out, 512, 1); run<8>(ncu, out, 1024, 1); run<8>(ncu, out, 1024, 2);
    return 0;
}
