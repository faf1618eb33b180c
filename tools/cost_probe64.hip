// cost_probe64.hip — issue cost of 64-bit VALU forms on gfx950 (round 2,
// session 3): can a SHA-256 rotate be a 64-bit shift of a duplicated word
// ({x, x} >> n = rotr(x, n) in the low half) at full rate, where
// v_alignbit_b32 issues at half rate (profiles/r02a_cost_probe.txt)?
//
//   hipcc --offload-arch=gfx950 -O3 -o build_exp/cost_probe64 tools/cost_probe64.hip && build_exp/cost_probe64
//
// Same harness as tools/cost_probe.hip part A: one 1024-thread workgroup per
// CU (4 waves/SIMD), 8 independent chains per wave, 64 instructions per
// iteration; cycles per wave64 instruction per SIMD at the in-kernel clock.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Stamp { unsigned long long t0, t1, r0, r1; };

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

#define PRE()                                                                              \
    extern __shared__ uint32_t tab[];                                                      \
    if (threadIdx.x == 0) tab[0] = seed;                                                   \
    __syncthreads();                                                                       \
    unsigned long long t0 = 0, r0 = 0;                                                     \
    if (threadIdx.x == 0) { t0 = memtime(); r0 = memrealtime(); }

#define POST(ACC)                                                                          \
    __syncthreads();                                                                       \
    if (threadIdx.x == 0) {                                                                \
        unsigned long long t1 = memtime(), r1 = memrealtime();                             \
        st[blockIdx.x].t0 = t0; st[blockIdx.x].t1 = t1; st[blockIdx.x].r0 = r0; st[blockIdx.x].r1 = r1; \
    }                                                                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(ACC) ^ (uint32_t)((ACC) >> 32);

// 64-bit chains: a_k are VGPR pairs, b a 32-bit VGPR, c a 64-bit VGPR pair
#define BODY8(INS)                                                                         \
    asm volatile(INS : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a1) : "v"(b), "v"(c)); \
    asm volatile(INS : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a3) : "v"(b), "v"(c)); \
    asm volatile(INS : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a5) : "v"(b), "v"(c)); \
    asm volatile(INS : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

#define KERNEL(NAME, INS)                                                                  \
    __global__ __launch_bounds__(1024) void NAME(uint32_t *out, Stamp *st, uint32_t seed, int iters) { \
        PRE()                                                                              \
        uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, c = seed * 5ull + threadIdx.x;     \
        uint32_t b = seed * 3;                                                             \
        asm volatile("" : "+v"(b), "+v"(c));                                               \
        for (int i = 0; i < iters; ++i) {                                                  \
            BODY8(INS) BODY8(INS) BODY8(INS) BODY8(INS)                                    \
            BODY8(INS) BODY8(INS) BODY8(INS) BODY8(INS)                                    \
        }                                                                                  \
        POST(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7)                                        \
    }

// 64-bit forms (32-bit references: v_xor_b32 2.40, v_alignbit_b32 4.26 cycles,
// profiles/r02a_cost_probe.txt)
KERNEL(k_lshr64, "v_lshrrev_b64 %0, 7, %0")
KERNEL(k_lshl64, "v_lshlrev_b64 %0, 7, %0")
KERNEL(k_lshr64_v, "v_lshrrev_b64 %0, %1, %0")
KERNEL(k_mov64, "v_mov_b64 %0, %2")
KERNEL(k_pkmov, "v_pk_mov_b32 %0, %0, %2 op_sel:[0,1]")
KERNEL(k_lshladd64, "v_lshl_add_u64 %0, %0, 1, %2")
KERNEL(k_pk_add_f32, "v_pk_add_f32 %0, %0, %2")

typedef void (*kfn)(uint32_t *, Stamp *, uint32_t, int);
static int ncu;
static uint32_t *d_out;
static Stamp *d_st;

static int run(const char *name, kfn k, int iters, double valu) {
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(ncu), dim3(1024), 131072, 0, d_out, d_st, 1u, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    double ghz = 0;
    unsigned long long cyc = 0;
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
            cyc = 0;
            for (int b = 0; b < ncu; ++b) {
                sum += (double)(h[b].t1 - h[b].t0) / (double)(h[b].r1 - h[b].r0) * 0.1;
                if (h[b].t1 - h[b].t0 > cyc) cyc = h[b].t1 - h[b].t0;
            }
            ghz = sum / ncu;
        }
    }
    printf("%-28s %8.3f ms  clk %.2f GHz  %9llu cyc  %.2f cyc/VALU/SIMD\n", name, best, ghz, cyc,
           cyc / (4.0 * valu * iters));
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
    printf("64 instr per iteration, 8 chains per wave, 4 waves/SIMD\n");
    run("lshrrev_b64 imm", k_lshr64, IA, 64);
    run("lshlrev_b64 imm", k_lshl64, IA, 64);
    run("lshrrev_b64 v", k_lshr64_v, IA, 64);
    run("mov_b64", k_mov64, IA, 64);
    run("pk_mov_b32", k_pkmov, IA, 64);
    run("lshl_add_u64", k_lshladd64, IA, 64);
    run("pk_add_f32", k_pk_add_f32, IA, 64);
    return 0;
}
