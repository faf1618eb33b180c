// rot_probe.hip — issue cost of the 32-bit rotate forms SHA-256 can use on
// gfx950: v_alignbit_b32 (x, x, n) against a 64-bit shift of the pair {x, x}
// (its low dword is rotr(x, n)), v_pk_mov_b32 (builds such a pair), and the
// full-rate references v_xor_b32 / v_bitop3_b32 / v_lshrrev_b32.  Each wave
// runs 8 independent chains of one instruction; 4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o build_tools/rot_probe tools/rot_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

enum Op { ALIGNBIT, SHR64, PKMOV, XOR, BITOP3, LSHR };

template <Op OP>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t seed, int iters) {
    uint64_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t x = threadIdx.x * (j + 3) ^ seed;
        v[j] = ((uint64_t)x << 32) | x;
    }
    uint32_t c = threadIdx.x * 13 + 1;
    asm volatile("" : "+v"(c));
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (OP == SHR64) {
                    asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(v[j]));
                } else if (OP == PKMOV) {
                    asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(v[j]));
                } else {
                    uint32_t lo = (uint32_t)v[j];
                    if (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(lo));
                    if (OP == XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(lo) : "v"(c));
                    if (OP == BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(lo) : "v"(c));
                    if (OP == LSHR) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(lo));
                    v[j] = (v[j] & 0xffffffff00000000ull) | lo;
                }
            }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= (uint32_t)v[j] ^ (uint32_t)(v[j] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <Op OP>
static int run(const char *name, int ncu, uint32_t *out) {
    const int iters = 4000;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k<OP>, dim3(ncu), dim3(1024), 0, 0, out, 1u, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k<OP>, dim3(ncu), dim3(1024), 0, 0, out, 2u + r, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double instr_per_simd = 4.0 * 64.0 * iters;     // 4 waves/SIMD x 64 instructions per iteration
    printf("%-18s %.3f ms  %.2f cyc/instr/SIMD @2.4GHz\n", name, best, best * 1e-3 * 2.4e9 / instr_per_simd);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    uint32_t *out;
    CHECK(hipMalloc(&out, 4ull * ncu * 1024));
    run<XOR>("v_xor_b32", ncu, out);
    run<BITOP3>("v_bitop3_b32", ncu, out);
    run<LSHR>("v_lshrrev_b32", ncu, out);
    run<ALIGNBIT>("v_alignbit_b32", ncu, out);
    run<SHR64>("v_lshrrev_b64", ncu, out);
    run<PKMOV>("v_pk_mov_b32", ncu, out);
    return 0;
}
