// cost_probe.hip — issue cost of the token kernels' instruction forms on gfx950,
// and whether LDS lookups and VALU work overlap when the waves that carry them
// share a SIMD (round-2 redo of overlap_probe.hip's confounded specialised case).
//
//   hipcc --offload-arch=gfx950 -O3 -o build_exp/cost_probe tools/cost_probe.hip && build_exp/cost_probe
//
// Every kernel: one workgroup of 1024 threads per CU (4 waves per SIMD; 128 KiB
// dynamic LDS pins one workgroup per CU, as the token kernels).  Wave 0 of
// every workgroup stamps s_memtime / s_memrealtime around the timed loop; the
// host reports the in-kernel clock and cycles per wave64 instruction per SIMD
// at THAT clock (not at 2.4 GHz).
//
// Part A — cost of one instruction form: 8 independent chains per wave, 64
// instructions per iteration.
// Part B — ds_read_b32 beside VALU in the same waves: 64 v_bitop3 plus N
// conflict-free lookups per iteration (the token kernels' replicated-table
// addressing, lane l on bank l&31), N = 0, 4, 8, 16.
// Part C — role split by hardware SIMD: each wave reads its SIMD id from
// HW_REG_HW_ID and takes a rank among the waves of that SIMD from an LDS
// counter; ranks 0-1 do only lookups (twice the per-wave share), ranks 2-3
// only VALU (twice the share): every SIMD carries both kinds of wave.  A
// second split puts lookups on SIMDs 0-1 and VALU on SIMDs 2-3.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef __attribute__((address_space(3))) const uint32_t l32;
typedef __attribute__((address_space(3))) uint32_t l32w;

struct Stamp { unsigned long long t0, t1, r0, r1; uint32_t simd_hist[4]; uint32_t pad[4]; };

__device__ __forceinline__ unsigned long long memtime() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long memrealtime() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ uint32_t simd_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    return (v >> 4) & 3u;
}

#define PRE()                                                                              \
    extern __shared__ uint32_t tab[];                                                      \
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) tab[i] = i * 2654435761u + seed; \
    __syncthreads();                                                                       \
    unsigned long long t0 = 0, r0 = 0;                                                     \
    if (threadIdx.x == 0) { t0 = memtime(); r0 = memrealtime(); }

#define POST(ACC)                                                                          \
    __syncthreads();                                                                       \
    if (threadIdx.x == 0) {                                                                \
        unsigned long long t1 = memtime(), r1 = memrealtime();                             \
        st[blockIdx.x].t0 = t0; st[blockIdx.x].t1 = t1; st[blockIdx.x].r0 = r0; st[blockIdx.x].r1 = r1; \
    }                                                                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (ACC);

// ---------------------------------------------------------------- part A --
#define BODY8(INS, B)                                                                      \
    asm volatile(INS : "+v"(a0) : B(b), "v"(c)); asm volatile(INS : "+v"(a1) : B(b), "v"(c)); \
    asm volatile(INS : "+v"(a2) : B(b), "v"(c)); asm volatile(INS : "+v"(a3) : B(b), "v"(c)); \
    asm volatile(INS : "+v"(a4) : B(b), "v"(c)); asm volatile(INS : "+v"(a5) : B(b), "v"(c)); \
    asm volatile(INS : "+v"(a6) : B(b), "v"(c)); asm volatile(INS : "+v"(a7) : B(b), "v"(c));

#define KERNEL(NAME, INS, B)                                                               \
    __global__ __launch_bounds__(1024) void NAME(uint32_t *out, Stamp *st, uint32_t seed, int iters) { \
        PRE()                                                                              \
        uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3, c = seed * 5 + threadIdx.x; \
        asm volatile("" : "+" B(b), "+v"(c));                                              \
        for (int i = 0; i < iters; ++i) {                                                  \
            BODY8(INS, B) BODY8(INS, B) BODY8(INS, B) BODY8(INS, B)                        \
            BODY8(INS, B) BODY8(INS, B) BODY8(INS, B) BODY8(INS, B)                        \
        }                                                                                  \
        POST(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7)                                        \
    }

KERNEL(k_bitop3_v, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
KERNEL(k_bitop3_s, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "s")
KERNEL(k_xor_v, "v_xor_b32 %0, %1, %0", "v")
KERNEL(k_xor_s, "v_xor_b32 %0, %1, %0", "s")
KERNEL(k_add_v, "v_add_u32 %0, %1, %0", "v")
KERNEL(k_add_lit, "v_add_u32 %0, 0x428a2f98, %0", "v")
KERNEL(k_add3_v, "v_add3_u32 %0, %0, %1, %2", "v")
KERNEL(k_add3_s, "v_add3_u32 %0, %0, %1, %2", "s")
KERNEL(k_perm_v, "v_perm_b32 %0, %0, %2, %1", "v")
KERNEL(k_perm_s, "v_perm_b32 %0, %0, %2, %1", "s")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %0, 7", "v")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 9, %0", "v")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 8, %2", "v")
KERNEL(k_and_or_v, "v_and_or_b32 %0, %0, %1, %2", "v")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, 8, 8", "v")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 8, %2", "v")
KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2", "v")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1", "v")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %2, vcc", "v")
KERNEL(k_mov_dpp, "v_mov_b32_dpp %0, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v")
KERNEL(k_alignbit_s, "v_alignbit_b32 %0, %0, %0, %1", "s")
// SDWA (round 2b): a byte of one register written into byte 1 of another,
// the other bytes preserved: a T-table address (byte << 8 | lane) in one op
KERNEL(k_sdwa_mov, "v_mov_b32_sdwa %0, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2", "v")
KERNEL(k_sdwa_mov_self, "v_mov_b32_sdwa %0, %0 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2", "v")
KERNEL(k_sdwa_mov_pad, "v_mov_b32_sdwa %0, %0 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_2", "v")
KERNEL(k_sdwa_xor, "v_xor_b32_sdwa %0, %0, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD", "v")

// ---------------------------------------------------------------- part B --
// 64 v_bitop3 (8 chains) plus NL lookups per iteration; the lookups' results
// fold into 4 sinks with v_bitop3 (NL/2 more VALU, counted).
template <int NL>
__global__ __launch_bounds__(1024) void k_mix(uint32_t *out, Stamp *st, uint32_t seed, int iters) {
    PRE()
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, b = seed * 3, c = seed * 5 + threadIdx.x;
    asm volatile("" : "+v"(b), "+v"(c));
    const uint32_t lane = 4u * (threadIdx.x & 31u);
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    uint32_t addr[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) addr[j] = (((threadIdx.x * 977u + j * 131u) & 0xffu) << 8) | lane | ((j & 1) << 16);
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(addr[j]));
    for (int i = 0; i < iters; ++i) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < NL; ++j) asm volatile("" : "+v"(addr[j]));   // no hoisting out of the loop
#pragma unroll
        for (int j = 0; j < NL; ++j) v[j] = *(l32 *)(uintptr_t)addr[j];
        BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
        BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
        BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
        BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
#pragma unroll
        for (int j = 0; j + 1 < NL; j += 8) {
            s0 = __builtin_amdgcn_bitop3_b32(s0, v[j], v[j + 1], 0x96);
            s1 = __builtin_amdgcn_bitop3_b32(s1, v[j + 2], v[j + 3], 0x96);
            s2 = __builtin_amdgcn_bitop3_b32(s2, v[j + 4], v[j + 5], 0x96);
            s3 = __builtin_amdgcn_bitop3_b32(s3, v[j + 6], v[j + 7], 0x96);
        }
        if (NL == 4) { s0 = __builtin_amdgcn_bitop3_b32(s0, v[0], v[1], 0x96); s1 = __builtin_amdgcn_bitop3_b32(s1, v[2], v[3], 0x96); }
    }
    POST(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ s1 ^ s2 ^ s3)
}

// LDS only: NL lookups per iteration, sinks as above (no other VALU).
template <int NL>
__global__ __launch_bounds__(1024) void k_ldsonly(uint32_t *out, Stamp *st, uint32_t seed, int iters) {
    PRE()
    const uint32_t lane = 4u * (threadIdx.x & 31u);
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    uint32_t addr[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) addr[j] = (((threadIdx.x * 977u + j * 131u) & 0xffu) << 8) | lane | ((j & 1) << 16);
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(addr[j]));
    for (int i = 0; i < iters; ++i) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < NL; ++j) asm volatile("" : "+v"(addr[j]));   // no hoisting out of the loop
#pragma unroll
        for (int j = 0; j < NL; ++j) v[j] = *(l32 *)(uintptr_t)addr[j];
#pragma unroll
        for (int j = 0; j + 1 < NL; j += 8) {
            s0 = __builtin_amdgcn_bitop3_b32(s0, v[j], v[j + 1], 0x96);
            s1 = __builtin_amdgcn_bitop3_b32(s1, v[j + 2], v[j + 3], 0x96);
            s2 = __builtin_amdgcn_bitop3_b32(s2, v[j + 4], v[j + 5], 0x96);
            s3 = __builtin_amdgcn_bitop3_b32(s3, v[j + 6], v[j + 7], 0x96);
        }
    }
    POST(s0 ^ s1 ^ s2 ^ s3)
}

// ---------------------------------------------------------------- part C --
// MODE 0: role by rank within the wave's hardware SIMD (2 lookup + 2 VALU waves
// per SIMD).  MODE 1: lookups on SIMDs 0-1, VALU on SIMDs 2-3.
// Lookup waves do 2 x 16 lookups per iteration (+16 sink ops), VALU waves 2 x 64 v_bitop3:
// the same total as k_mix<16> run by every wave.
template <int MODE>
__global__ __launch_bounds__(1024) void k_split(uint32_t *out, Stamp *st, uint32_t seed, int iters) {
    extern __shared__ uint32_t tab[];
    l32w *cnt = (l32w *)(uintptr_t)(131072 - 64);
    for (int i = threadIdx.x; i < 32768 - 16; i += blockDim.x) tab[i] = i * 2654435761u + seed;
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t simd = simd_id();
    uint32_t rank = 0;
    if ((threadIdx.x & 63u) == 0) rank = __hip_atomic_fetch_add(&cnt[simd], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    rank = __builtin_amdgcn_readfirstlane(rank);
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) st[blockIdx.x].simd_hist[k] = cnt[k];
    }
    const bool lds_role = MODE == 0 ? rank < 2u : simd < 2u;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = memtime(); r0 = memrealtime(); }
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, b = seed * 3, c = seed * 5 + threadIdx.x;
    asm volatile("" : "+v"(b), "+v"(c));
    const uint32_t lane = 4u * (threadIdx.x & 31u);
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    uint32_t addr[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) addr[j] = (((threadIdx.x * 977u + j * 131u) & 0xffu) << 8) | lane | ((j & 1) << 16);
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(addr[j]));
    if (lds_role) {
        for (int i = 0; i < 2 * iters; ++i) {
            uint32_t v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(addr[j]));
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = *(l32 *)(uintptr_t)addr[j];
#pragma unroll
            for (int j = 0; j < 16; j += 8) {
                s0 = __builtin_amdgcn_bitop3_b32(s0, v[j], v[j + 1], 0x96);
                s1 = __builtin_amdgcn_bitop3_b32(s1, v[j + 2], v[j + 3], 0x96);
                s2 = __builtin_amdgcn_bitop3_b32(s2, v[j + 4], v[j + 5], 0x96);
                s3 = __builtin_amdgcn_bitop3_b32(s3, v[j + 6], v[j + 7], 0x96);
            }
        }
    } else {
        for (int i = 0; i < 2 * iters; ++i) {
            BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
            BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
            BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
            BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v") BODY8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", "v")
        }
    }
    POST(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ s1 ^ s2 ^ s3)
}

// ------------------------------------------------------------------ host --
typedef void (*kfn)(uint32_t *, Stamp *, uint32_t, int);

static int ncu;
static uint32_t *d_out;
static Stamp *d_st;

// valu: wave64 VALU instructions per wave per iteration; lds: ds_read per wave per iteration
static int run(const char *name, kfn k, int iters, double valu, double lds, bool hist = false) {
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(ncu), dim3(1024), 131072, 0, d_out, d_st, 1u, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    double ghz = 0;
    Stamp *h = (Stamp *)malloc(sizeof(Stamp) * ncu);
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k, dim3(ncu), dim3(1024), 131072, 0, d_out, d_st, 2u + r, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) {
            best = ms;
            CHECK(hipMemcpy(h, d_st, sizeof(Stamp) * ncu, hipMemcpyDeviceToHost));
            double sum = 0;
            for (int b = 0; b < ncu; ++b) sum += (double)(h[b].t1 - h[b].t0) / (double)(h[b].r1 - h[b].r0) * 0.1;
            ghz = sum / ncu;
        }
    }
    // in-kernel cycles of the slowest workgroup
    unsigned long long cyc = 0;
    for (int b = 0; b < ncu; ++b) cyc = (h[b].t1 - h[b].t0) > cyc ? (h[b].t1 - h[b].t0) : cyc;
    const double per_simd_valu = 4.0 * valu * iters, per_cu_lds = 16.0 * lds * iters;
    printf("%-28s %8.3f ms  clk %.2f GHz  %9llu cyc", name, best, ghz, cyc);
    if (valu > 0) printf("  %.2f cyc/VALU/SIMD", cyc / per_simd_valu);
    if (lds > 0) printf("  %.2f cyc/ds_read/CU", cyc / per_cu_lds);
    if (hist) printf("  waves/SIMD %u %u %u %u", h[0].simd_hist[0], h[0].simd_hist[1], h[0].simd_hist[2], h[0].simd_hist[3]);
    printf("\n");
    free(h);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    ncu = p.multiProcessorCount;
    CHECK(hipMalloc(&d_out, 4ull * ncu * 1024));
    CHECK(hipMalloc(&d_st, sizeof(Stamp) * ncu));
    const int IA = 4000;
    printf("part A: 64 instr per iteration, 8 chains per wave, 4 waves/SIMD\n");
    run("bitop3 v,v,v", k_bitop3_v, IA, 64, 0);
    run("bitop3 v,s,v", k_bitop3_s, IA, 64, 0);
    run("xor v,v", k_xor_v, IA, 64, 0);
    run("xor s,v", k_xor_s, IA, 64, 0);
    run("add_u32 v,v", k_add_v, IA, 64, 0);
    run("add_u32 literal,v", k_add_lit, IA, 64, 0);
    run("add3 v,v,v", k_add3_v, IA, 64, 0);
    run("add3 v,s,v", k_add3_s, IA, 64, 0);
    run("perm v,v,v(sel)", k_perm_v, IA, 64, 0);
    run("perm v,v,s(sel)", k_perm_s, IA, 64, 0);
    run("alignbit v,v,imm", k_alignbit, IA, 64, 0);
    run("alignbit v,v,s", k_alignbit_s, IA, 64, 0);
    run("lshrrev imm", k_lshr, IA, 64, 0);
    run("lshl_or v,imm,v", k_lshl_or, IA, 64, 0);
    run("and_or v,v,v", k_and_or_v, IA, 64, 0);
    run("bfe_u32 v,imm,imm", k_bfe, IA, 64, 0);
    run("lshl_add v,imm,v", k_lshl_add, IA, 64, 0);
    run("mad_u32_u24 v,v,v", k_mad_u24, IA, 64, 0);
    run("pk_add_u16 v,v", k_pk_add_u16, IA, 64, 0);
    run("cndmask v,v,vcc", k_cndmask, IA, 64, 0);
    run("mov_dpp quad_perm", k_mov_dpp, IA, 64, 0);
    run("mov_sdwa byte2->byte1 preserve", k_sdwa_mov, IA, 64, 0);
    run("mov_sdwa self preserve", k_sdwa_mov_self, IA, 64, 0);
    run("mov_sdwa self pad", k_sdwa_mov_pad, IA, 64, 0);
    run("xor_sdwa src0 byte2", k_sdwa_xor, IA, 64, 0);
    const int IB = 4000;
    printf("part B: 64 bitop3 + N ds_read_b32 (+N/2 sink bitop3) in every wave\n");
    run("mix N=0", k_mix<0>, IB, 64, 0);
    run("mix N=4", k_mix<4>, IB, 66, 4);
    run("mix N=8", k_mix<8>, IB, 68, 8);
    run("mix N=16", k_mix<16>, IB, 72, 16);
    run("lds only N=16", k_ldsonly<16>, IB, 8, 16);
    run("lds only N=8", k_ldsonly<8>, IB, 4, 8);
    printf("part C: same work as mix N=16, roles split across waves\n");
    run("split by rank within SIMD", k_split<0>, IB, 72, 16, true);
    run("split SIMD 0-1 | 2-3", k_split<1>, IB, 72, 16, true);
    return 0;
}
