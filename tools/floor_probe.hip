// floor_probe.hip — how much of the c2 kernels' time is their compute core?
//
// The issue-cost model of DESIGN.md §4.5 prices the hot loop's instruction mix
// with per-form costs from tools/cost_probe.hip and finds k_encrypt<14,false>
// at ~84 % of that floor.  This probe measures the floor directly instead of
// pricing it: the kernels' own device code (enc_quad / dec_quad /
// sha256_compress from token_device.h, the same inlining and compiler
// schedule) run in register-only loops, with no global loads or stores, no
// packet loop and no tail handling, at the launch shape of c2 (one 1024- or
// 768-thread workgroup per CU, the 128 / 160 KiB table image).
//
//   core_enc   : enc_quad<14, true> per iteration (4 CBC blocks + the SHA-256
//                compression of the previous quad), the ciphertext fed back
//                as the next plaintext and as the next SHA block
//   core_enc0  : enc_quad<14, false> (quad 0 of a packet: AES chain only)
//   core_dec   : dec_quad<14, true> (4 independent blocks + one compression),
//                at 768 threads (the c2 kernel's shape) and at 1024
//   core_sha   : sha256_compress alone (hmac_finish's compressions)
//   core_enc_x2: two packets per lane (two CBC chains and two compressions
//                interleaved round by round) at 512 threads = 2 waves/SIMD,
//                round keys in SGPRs or (x2vk) in VGPRs
//
// Per c2 wave-packet (64 packets of 500 B): encrypt = 1 x core_enc0 + 7 x
// core_enc + 3 x core_sha; decrypt = 8 x core_dec + 2 x core_sha.  The host
// prints SIMD-cycles per wave-iteration (in-kernel s_memtime cycles / waves
// per SIMD / iterations) and that per-packet sum, to set beside the kernel's
// GRBM_GUI_ACTIVE per wave-packet (profiles/r02y_pmc_summary.txt).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build_exp/floor_probe tools/floor_probe.hip && build_exp/floor_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../reticulum_amd/csrc/token_device.h"

using namespace rnstok;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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

// Table image: contents do not matter for timing (any 32-bit values), only
// the footprint and the conflict-free addressing of token_device.h.
__device__ void fill_any(uint32_t *tab, uint32_t words, uint32_t seed) {
    for (uint32_t d = threadIdx.x; d < words; d += blockDim.x) tab[d] = d * 2654435761u + seed;
    __syncthreads();
}

#define STAMP_BEGIN()                                                                      \
    unsigned long long t0 = 0, r0 = 0;                                                     \
    if (threadIdx.x == 0) { t0 = memtime(); r0 = memrealtime(); }
#define STAMP_END(ACC)                                                                     \
    __syncthreads();                                                                       \
    if (threadIdx.x == 0) {                                                                \
        unsigned long long t1 = memtime(), r1 = memrealtime();                             \
        st[blockIdx.x].t0 = t0; st[blockIdx.x].t1 = t1; st[blockIdx.x].r0 = r0; st[blockIdx.x].r1 = r1; \
    }                                                                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (ACC);

template <bool WITH_SHA>
__global__ __launch_bounds__(1024) void k_core_enc(const uint32_t *rec, uint32_t *out, Stamp *st, uint32_t seed, int iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    fill_any(tab, LDS_ENC_BYTES / 4, seed);
    const Lanes LN(threadIdx.x & 31u);
    uint32_t rk[60];
#pragma unroll
    for (int i = 0; i < 60; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rec[i]);
    const uint32_t t = threadIdx.x * 0x9E3779B9u ^ seed;
    u32x4 x[4], c[4], prev = {t, t + 1, t + 2, t + 3};
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = u32x4{t ^ j, t + 7 * j, t * 3 + j, t ^ (j << 9)};
    Sha256 S;
#pragma unroll
    for (int k = 0; k < 16; ++k) S.w[k] = t + k;
    uint32_t h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = rk[k] ^ t;
    STAMP_BEGIN()
#pragma nounroll
    for (int i = 0; i < iters; ++i) {
        if (WITH_SHA) S.start(h);
        enc_quad<14, WITH_SHA>(c, x, prev, rk, LN, S);
        if (WITH_SHA) {
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(S.v[k]));
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] += S.v[k];
            sha_units(S.w, prev, c[0], c[1], c[2]);
        }
        prev = c[3];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = c[j] ^ x[j];   // next "plaintext": depends on this quad
    }
    uint32_t acc = prev.x ^ prev.y ^ prev.z ^ prev.w;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= h[k];
    STAMP_END(acc)
}

// Two packets per lane, their CBC chains and SHA rounds interleaved round by
// round (ILP inside the wave instead of across waves), at 2 waves/SIMD; the
// round keys in SGPRs (VK = false) or in VGPRs (VK = true: 256 VGPRs allow it).
template <int NR, bool VK>
__device__ __forceinline__ void enc_quad_x2(u32x4 c[2][4], const u32x4 x[2][4], const u32x4 chain[2],
                                            const uint32_t *rk, const Lanes &L, Sha256 S[2]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        uint32_t st[2][4];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const u32x4 in = x[k][b] ^ (b == 0 ? chain[k] : c[k][b - 1]);
            st[k][0] = in.x ^ rk[0]; st[k][1] = in.y ^ rk[1]; st[k][2] = in.z ^ rk[2]; st[k][3] = in.w ^ rk[3];
        }
#pragma unroll
        for (int r = 1; r < NR; ++r) {
            uint32_t v[2][16];
            tround_load<false>(v[0], st[0], L);
            tround_load<false>(v[1], st[1], L);
            S[0].round(b * NR + r - 1);
            S[1].round(b * NR + r - 1);
            tround_mix(st[0], v[0], rk + 4 * r);
            tround_mix(st[1], v[1], rk + 4 * r);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t s0 = st[k][0], s1 = st[k][1], s2 = st[k][2], s3 = st[k][3];
            c[k][b].x = tlast_enc(s0, s1, s2, s3, rk[4 * NR + 0], L);
            c[k][b].y = tlast_enc(s1, s2, s3, s0, rk[4 * NR + 1], L);
            c[k][b].z = tlast_enc(s2, s3, s0, s1, rk[4 * NR + 2], L);
            c[k][b].w = tlast_enc(s3, s0, s1, s2, rk[4 * NR + 3], L);
            S[k].round(b * NR + NR - 1);
        }
    }
#pragma unroll
    for (int i = 4 * NR; i < 64; ++i) {
        S[0].round(i);
        S[1].round(i);
    }
}

template <bool VK>
__global__ __launch_bounds__(512) void k_core_enc_x2(const uint32_t *rec, uint32_t *out, Stamp *st, uint32_t seed, int iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    fill_any(tab, LDS_ENC_BYTES / 4, seed);
    const Lanes LN(threadIdx.x & 31u);
    uint32_t rk[60];
#pragma unroll
    for (int i = 0; i < 60; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rec[i]);
    if (VK) {
#pragma unroll
        for (int i = 0; i < 60; ++i) asm volatile("" : "+v"(rk[i]));
    }
    const uint32_t t = threadIdx.x * 0x9E3779B9u ^ seed;
    u32x4 x[2][4], c[2][4], prev[2];
    Sha256 S[2];
    uint32_t h[2][8];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t tk = t + 0x1234567u * k;
        prev[k] = u32x4{tk, tk + 1, tk + 2, tk + 3};
#pragma unroll
        for (int j = 0; j < 4; ++j) x[k][j] = u32x4{tk ^ j, tk + 7 * j, tk * 3 + j, tk ^ (j << 9)};
#pragma unroll
        for (int i = 0; i < 16; ++i) S[k].w[i] = tk + i;
#pragma unroll
        for (int i = 0; i < 8; ++i) h[k][i] = rk[i] ^ tk;
    }
    STAMP_BEGIN()
#pragma nounroll
    for (int i = 0; i < iters; ++i) {
        S[0].start(h[0]);
        S[1].start(h[1]);
        enc_quad_x2<14, VK>(c, x, prev, rk, LN, S);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(S[k].v[j]));
#pragma unroll
            for (int j = 0; j < 8; ++j) h[k][j] += S[k].v[j];
            sha_units(S[k].w, prev[k], c[k][0], c[k][1], c[k][2]);
            prev[k] = c[k][3];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[k][j] = c[k][j] ^ x[k][j];
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        acc ^= prev[k].x ^ prev[k].w;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= h[k][j];
    }
    STAMP_END(acc)
}

template <int WG>
__global__ __launch_bounds__(WG) void k_core_dec(const uint32_t *rec, uint32_t *out, Stamp *st, uint32_t seed, int iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    fill_any(tab, LDS_DEC_BYTES / 4, seed);
    const Lanes LN(threadIdx.x & 31u);
    uint32_t rk[60];
#pragma unroll
    for (int i = 0; i < 60; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rec[i]);
    const uint32_t t = threadIdx.x * 0x9E3779B9u ^ seed;
    u32x4 c[4], pp[4], prev = {t, t + 1, t + 2, t + 3};
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = u32x4{t ^ j, t + 7 * j, t * 3 + j, t ^ (j << 9)};
    Sha256 S;
    uint32_t h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = rk[k] ^ t;
    STAMP_BEGIN()
#pragma nounroll
    for (int i = 0; i < iters; ++i) {
        S.start(h);
        sha_units(S.w, prev, c[0], c[1], c[2]);
        dec_quad<14, true>(pp, c, prev, rk, LN, S);
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(S.v[k]));
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] += S.v[k];
        prev = c[3];
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = c[j] ^ pp[j];   // next "ciphertext": depends on this quad
    }
    uint32_t acc = prev.x ^ prev.y ^ prev.z ^ prev.w;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= h[k];
    STAMP_END(acc)
}

__global__ __launch_bounds__(1024) void k_core_sha(const uint32_t *rec, uint32_t *out, Stamp *st, uint32_t seed, int iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    fill_any(tab, LDS_ENC_BYTES / 4, seed);
    const uint32_t t = threadIdx.x * 0x9E3779B9u ^ seed;
    uint32_t h[8], w[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = rec[k] ^ t;
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = t + 3 * k;
    STAMP_BEGIN()
#pragma nounroll
    for (int i = 0; i < iters; ++i) {
        sha256_compress(h, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] ^= h[k];          // next block depends on this one
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= h[k];
    STAMP_END(acc)
}

// Split roles: waves [0, AW) run the AES chain alone
// (enc_quad<14, false>, `iters` quads each), waves [AW, 16) the SHA-256
// compressions alone (iters * AW / (16 - AW) each), so the SIMDs carry the
// same work as k_core_enc's 16 x iters mixed quads.  Wave w sits on SIMD w % 4.
template <int AW>
__global__ __launch_bounds__(1024) void k_core_split(const uint32_t *rec, uint32_t *out, Stamp *st, uint32_t seed,
                                                     int iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    fill_any(tab, LDS_ENC_BYTES / 4, seed);
    const Lanes LN(threadIdx.x & 31u);
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t t = threadIdx.x * 0x9E3779B9u ^ seed;
    uint32_t acc = 0;
    STAMP_BEGIN()
    if (wave < (uint32_t)AW) {
        uint32_t rk[60];
#pragma unroll
        for (int i = 0; i < 60; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rec[i]);
        u32x4 x[4], c[4], prev = {t, t + 1, t + 2, t + 3};
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = u32x4{t ^ j, t + 7 * j, t * 3 + j, t ^ (j << 9)};
        Sha256 S;
#pragma nounroll
        for (int i = 0; i < iters; ++i) {
            enc_quad<14, false>(c, x, prev, rk, LN, S);
            prev = c[3];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = c[j] ^ x[j];
        }
        acc = prev.x ^ prev.y ^ prev.z ^ prev.w;
    } else {
        uint32_t h[8], w[16];
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = rec[k] ^ t;
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = t + 3 * k;
        const int n = iters * AW / (16 - AW);
#pragma nounroll
        for (int i = 0; i < n; ++i) {
            sha256_compress(h, w);
#pragma unroll
            for (int k = 0; k < 8; ++k) w[k] ^= h[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= h[k];
    }
    STAMP_END(acc)
}

// The same split for decryption: waves [0, AW) dec_quad<14, false> (4
// independent blocks, no SHA), waves [AW, 16) the compressions.
template <int AW>
__global__ __launch_bounds__(1024) void k_core_dsplit(const uint32_t *rec, uint32_t *out, Stamp *st, uint32_t seed,
                                                      int iters) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    fill_any(tab, LDS_DEC_BYTES / 4, seed);
    const Lanes LN(threadIdx.x & 31u);
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t t = threadIdx.x * 0x9E3779B9u ^ seed;
    uint32_t acc = 0;
    STAMP_BEGIN()
    if (wave < (uint32_t)AW) {
        uint32_t rk[60];
#pragma unroll
        for (int i = 0; i < 60; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rec[i]);
        u32x4 c[4], pp[4], prev = {t, t + 1, t + 2, t + 3};
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = u32x4{t ^ j, t + 7 * j, t * 3 + j, t ^ (j << 9)};
        Sha256 S;
#pragma nounroll
        for (int i = 0; i < iters; ++i) {
            dec_quad<14, false>(pp, c, prev, rk, LN, S);
            prev = c[3];
#pragma unroll
            for (int j = 0; j < 4; ++j) c[j] = c[j] ^ pp[j];
        }
        acc = prev.x ^ prev.y ^ prev.z ^ prev.w;
    } else {
        uint32_t h[8], w[16];
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = rec[k] ^ t;
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = t + 3 * k;
        const int n = iters * AW / (16 - AW);
#pragma nounroll
        for (int i = 0; i < n; ++i) {
            sha256_compress(h, w);
#pragma unroll
            for (int k = 0; k < 8; ++k) w[k] ^= h[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= h[k];
    }
    STAMP_END(acc)
}

typedef void (*kfn)(const uint32_t *, uint32_t *, Stamp *, uint32_t, int);
static int ncu;
static uint32_t *d_out, *d_rec;
static Stamp *d_st;

// returns SIMD-cycles per wave-iteration (slowest workgroup)
static double run(const char *name, kfn k, int threads, uint32_t lds, int iters) {
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(ncu), dim3(threads), lds, 0, d_rec, d_out, d_st, 1u, iters);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    double ghz = 0;
    unsigned long long cyc = 0;
    Stamp *h = (Stamp *)malloc(sizeof(Stamp) * ncu);
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k, dim3(ncu), dim3(threads), lds, 0, d_rec, d_out, d_st, 2u + r, iters);
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
    const double waves_per_simd = threads / 64 / 4.0;
    const double per = cyc / waves_per_simd / iters;
    printf("%-12s %4d thr  %8.3f ms  clk %.2f GHz  %10llu cyc  %8.0f SIMD-cycles per wave-iteration\n", name, threads,
           best, ghz, cyc, per);
    free(h);
    return per;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    ncu = p.multiProcessorCount;
    CHECK(hipMalloc(&d_out, 4ull * ncu * 1024));
    CHECK(hipMalloc(&d_rec, 4ull * 136));
    CHECK(hipMemset(d_rec, 0x5a, 4ull * 136));
    CHECK(hipMalloc(&d_st, sizeof(Stamp) * ncu));
    const int IQ = 400, IS = 2000;
    const double qe = run("core_enc", k_core_enc<true>, 1024, LDS_ENC_BYTES, IQ);
    const double q0 = run("core_enc0", k_core_enc<false>, 1024, LDS_ENC_BYTES, IQ);
    const double qd = run("core_dec", k_core_dec<768>, 768, LDS_DEC_BYTES, IQ);
    run("core_dec", k_core_dec<1024>, 1024, LDS_DEC_BYTES, IQ);
    const double cs = run("core_sha", k_core_sha, 1024, LDS_ENC_BYTES, IS);
    // 2 packets per lane at 2 waves/SIMD: per-packet cost = cycles per wave-iteration / 2
    // split roles: per wave-iteration figures are per AES quad of the AES
    // waves; the SIMD carries AW/4 AES waves, so per mixed-quad-equivalent:
    // cycles * 4 waves / (AW/4 waves) ... printed as SIMD-cycles per quad+compression
    for (int aw : {8, 10, 12}) {
        kfn k = aw == 8 ? k_core_split<8> : (aw == 10 ? k_core_split<10> : k_core_split<12>);
        char nm[32];
        snprintf(nm, sizeof nm, "core_split%d", aw);
        const double per = run(nm, k, 1024, LDS_ENC_BYTES, IQ);
        printf("  split %d AES + %d SHA waves: %.0f SIMD-cycles per (AES quad + compression), mixed core_enc %.0f\n",
               aw, 16 - aw, per * 16.0 / aw, qe);
    }
    for (int aw : {8, 10, 12}) {
        kfn k = aw == 8 ? k_core_dsplit<8> : (aw == 10 ? k_core_dsplit<10> : k_core_dsplit<12>);
        char nm[32];
        snprintf(nm, sizeof nm, "core_dsplit%d", aw);
        const double per = run(nm, k, 1024, LDS_DEC_BYTES, IQ);
        printf("  dsplit %d AES + %d SHA waves: %.0f SIMD-cycles per (AES dec quad + compression), mixed core_dec %.0f\n",
               aw, 16 - aw, per * 16.0 / aw, qd);
    }
    const double x2s = run("core_enc_x2", k_core_enc_x2<false>, 512, LDS_ENC_BYTES, IQ);
    const double x2v = run("core_enc_x2vk", k_core_enc_x2<true>, 512, LDS_ENC_BYTES, IQ);
    printf("two packets per lane: %.0f (SGPR keys) / %.0f (VGPR keys) SIMD-cycles per packet-quad, against %.0f\n",
           x2s / 2, x2v / 2, qe);
    printf("per c2 wave-packet (64 x 500 B): encrypt core %.0f SIMD-cycles (q0 + 7 q + 3 sha), "
           "decrypt core %.0f (8 q + 2 sha)\n", q0 + 7 * qe + 3 * cs, 8 * qd + 2 * cs);
    printf("per SIMD per c2 launch (2^20 packets, %d CUs): encrypt core %.3f M cycles, decrypt core %.3f M cycles\n",
           ncu, (q0 + 7 * qe + 3 * cs) * (1048576.0 / 64 / (4 * ncu)) / 1e6,
           (8 * qd + 2 * cs) * (1048576.0 / 64 / (4 * ncu)) / 1e6);
    return 0;
}
