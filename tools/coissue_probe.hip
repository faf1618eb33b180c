// coissue_probe.hip — do LDS lookups and VALU work of different waves issue in
// the same cycles on gfx950?  (the split-role encrypt showed
// VALU + LDS slot-cycles at 1.10x its cycles; this measures the mechanism
// directly.)  One 1024-thread workgroup per CU (4 waves per SIMD), LDS table
// of 64 KiB, conflict-free ds_read_b32 (lane l reads bank l & 31):
//   lds    : every wave issues only table lookups (16 independent per step)
//   valu   : every wave issues only full-rate v_xor_b32 (16 independent per step)
//   perm   : every wave issues only v_perm_b32 (single-issue form)
//   mix    : waves 0-7 lookups, waves 8-15 v_xor (2 + 2 per SIMD), same per-wave work
//   mixp   : waves 0-7 lookups, waves 8-15 v_perm
// Per mode: cycles (wall of the launch x clock) per SIMD-step, where a
// SIMD-step is one step of each of the SIMD's four waves.  No co-issue:
// mix = (lds + valu) / 2; full co-issue: mix = max(lds, valu) / 2 ... per the
// four waves' shares; printed against both.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build_exp/coissue_probe tools/coissue_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int STEPS = 20000;

template <int MODE>   // 0 lds, 1 valu, 2 perm, 3 mix (lds | valu), 4 mixp (lds | perm)
__global__ __launch_bounds__(1024) void k_probe(uint32_t *out, uint32_t seed) {
    extern __shared__ uint32_t tab[];
    for (uint32_t i = threadIdx.x; i < 16384u; i += 1024u) tab[i] = i * 2654435761u + seed;
    __syncthreads();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 31u;
    const bool do_lds = MODE == 0 || ((MODE == 3 || MODE == 4) && wave < 8u);
    const bool do_perm = MODE == 2 || (MODE == 4 && wave >= 8u);
    uint32_t acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = seed + k * 77u + threadIdx.x;
    if (do_lds) {
        typedef __attribute__((address_space(3))) uint32_t lds_t;
        uint32_t addr[16];                                   // fixed, conflict-free: no VALU in the loop
#pragma unroll
        for (int k = 0; k < 16; ++k) addr[k] = 4u * lane + 128u * (uint32_t)(k * 37 & 127);
#pragma nounroll
        for (int s = 0; s < STEPS; ++s) {
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("ds_read_b32 %0, %1" : "=v"(acc[k]) : "v"(addr[k]) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    } else if (do_perm) {
        const uint32_t sel = 0x05040100u + seed * 0u;
#pragma nounroll
        for (int s = 0; s < STEPS; ++s) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(acc[k]) : "v"(acc[(k + 1) & 15]), "v"(sel));
        }
    } else {
#pragma nounroll
        for (int s = 0; s < STEPS; ++s) {
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc[k]) : "v"(acc[(k + 5) & 15]));
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) r ^= acc[k];
    if (r == 0x12345678u) out[blockIdx.x] = r;
}

template <int MODE>
static double run(int ncu, uint32_t *d_out) {
    auto k = k_probe<MODE>;
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    hipLaunchKernelGGL(k, dim3(ncu), dim3(1024), 65536, 0, d_out, 1u);      // warm
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    double best = 1e30;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k, dim3(ncu), dim3(1024), 65536, 0, d_out, 2u + r);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char **argv) {
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;      // the clock the cycles are quoted at
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    uint32_t *d_out;
    CHECK(hipMalloc(&d_out, 4 * ncu));
    const double ms[5] = {run<0>(ncu, d_out), run<1>(ncu, d_out), run<2>(ncu, d_out), run<3>(ncu, d_out),
                          run<4>(ncu, d_out)};
    const char *name[5] = {"lds", "valu", "perm", "mix(lds|valu)", "mixp(lds|perm)"};
    // per wave and step: 16 instructions; a SIMD-step = 4 waves x 16 instructions
    printf("%d CUs, %d steps, 16 instructions per wave-step, cycles at %.2f GHz\n", ncu, STEPS, ghz);
    for (int m = 0; m < 5; ++m)
        printf("%-16s %8.3f ms  %7.2f cycles per SIMD-step (64 instructions)\n", name[m], ms[m],
               ms[m] * 1e-3 * ghz * 1e9 / STEPS);
    printf("mix : no co-issue would be %.3f ms, full co-issue %.3f ms\n", (ms[0] + ms[1]) / 2,
           (ms[0] > ms[1] ? ms[0] : ms[1]) / 2);
    printf("mixp: no co-issue would be %.3f ms, full co-issue %.3f ms\n", (ms[0] + ms[2]) / 2,
           (ms[0] > ms[2] ? ms[0] : ms[2]) / 2);
    return 0;
}
