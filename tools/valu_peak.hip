// valu_peak.hip — measured issue rates of the integer VALU / LDS instructions
// the token kernels are built from, on the whole chip (all CUs busy).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_peak tools/valu_peak.hip && build/valu_peak
//
// Each kernel runs 8 independent chains of one instruction per lane so the
// result is throughput, not latency.  Prints lane-ops/s and cycles per wave64
// instruction per SIMD at the measured clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

#define BODY8(INS)                                                                         \
    asm volatile(INS : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a1) : "v"(b), "v"(c)); \
    asm volatile(INS : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a3) : "v"(b), "v"(c)); \
    asm volatile(INS : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a5) : "v"(b), "v"(c)); \
    asm volatile(INS : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

#define KERNEL(NAME, INS)                                                                  \
    __global__ __launch_bounds__(1024) void NAME(uint32_t *out, uint32_t seed) {           \
        uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3, c = seed * 5 + 1;     \
        for (int i = 0; i < ITERS; ++i) { BODY8(INS) BODY8(INS) }                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }

KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, %2")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_fma, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_sdwa_mov, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2")
KERNEL(k_sdwa_and, "v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3 src1_sel:DWORD")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, %1, %2")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, %1, %2")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, %1, %2")
KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, %2")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_lshr, "v_lshrrev_b32 %0, %1, %0")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_add_co, "v_add_co_u32 %0, vcc, %0, %1")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")

// ds_read_b32 throughput with the token kernels' replicated-table pattern:
// lane l reads bank (l & 31) of a random 256-B row.
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out, uint32_t seed) {
    extern __shared__ uint32_t tab[];
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) tab[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lc = 4u * (threadIdx.x & 31u);
    uint32_t x0 = threadIdx.x * 977u ^ seed, x1 = x0 * 3u, x2 = x0 * 5u, x3 = x0 * 7u;
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t a0 = __builtin_amdgcn_perm(x0, lc, 0x0C0C0400u), a1 = __builtin_amdgcn_perm(x1, lc, 0x0C0C0500u);
            const uint32_t a2 = __builtin_amdgcn_perm(x2, lc, 0x0C0C0600u), a3 = __builtin_amdgcn_perm(x3, lc, 0x0C0C0700u);
            typedef __attribute__((address_space(3))) const uint32_t l32;
            x0 ^= *(l32 *)(uintptr_t)a0; x1 ^= *(l32 *)(uintptr_t)(a1 + 128);
            x2 ^= *(l32 *)(uintptr_t)(a2 + 0x8000); x3 ^= *(l32 *)(uintptr_t)(a3 + 0x8080);
        }
        acc += x0 ^ x1 ^ x2 ^ x3;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    int dev = 0;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, dev));
    const int ncu = p.multiProcessorCount;
    const int blocks = ncu * 2, threads = 1024;   // 8 waves per SIMD worth of work, 2 blocks per CU over time
    uint32_t *out;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * threads));
    CHECK(hipFuncSetAttribute((const void *)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct { const char *name; void (*k)(uint32_t *, uint32_t); double per_iter; size_t lds; } ks[] = {
        {"v_add_u32", k_add, 16, 0}, {"v_xor_b32", k_xor, 16, 0}, {"v_perm_b32", k_perm, 16, 0},
        {"v_alignbit_b32", k_alignbit, 16, 0}, {"v_bitop3_b32", k_bitop3, 16, 0}, {"v_add3_u32", k_add3, 16, 0},
        {"v_bfi_b32", k_bfi, 16, 0}, {"v_fma_f32", k_fma, 16, 0},
        {"v_mov_b32_sdwa", k_sdwa_mov, 16, 0}, {"v_and_b32_sdwa", k_sdwa_and, 16, 0},
        {"v_and_or_b32", k_and_or, 16, 0}, {"v_lshl_or_b32", k_lshl_or, 16, 0}, {"v_lshl_add_u32", k_lshl_add, 16, 0},
        {"v_bfe_u32", k_bfe, 16, 0}, {"v_alignbyte_b32", k_alignbyte, 16, 0}, {"v_xad_u32", k_xad, 16, 0},
        {"v_lshrrev_b32", k_lshr, 16, 0}, {"v_pk_add_u16", k_pk_add_u16, 16, 0}, {"v_add_co_u32", k_add_co, 16, 0},
        {"v_or3_b32", k_or3, 16, 0}, {"ds_read_b32(lookup)", k_lds, 16, 131072},
    };
    printf("CUs %d, clock spec %.0f MHz\n", ncu, p.clockRate / 1000.0);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), k.lds, 0, out, 1u);   // warm-up
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CHECK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), k.lds, 0, out, 2u + r);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const double lane_ops = (double)blocks * threads * ITERS * k.per_iter;
        const double rate = lane_ops / (best * 1e-3);
        // wave64 instructions per SIMD, cycles at 2.4 GHz
        const double wave_instr_per_simd = lane_ops / 64.0 / (ncu * 4.0);
        printf("%-22s %8.3f ms  %7.2f T lane-op/s  %5.2f cyc/wave-instr/SIMD @2.4GHz  (%.1f%% of CUs*128*2.4G)\n",
               k.name, best, rate / 1e12, best * 1e-3 * 2.4e9 / wave_instr_per_simd,
               100.0 * rate / (ncu * 128.0 * 2.4e9));
    }
    return 0;
}
