// split_probe.hip — would splitting Token.encrypt into an AES-CBC kernel and an
// HMAC-SHA256 kernel that run CONCURRENTLY on the same CUs beat the fused
// kernel?  The AES kernel is LDS-bound (128 KiB table image, 16 waves/CU); the
// HMAC kernel needs no LDS and is pure VALU, so both can be co-resident
// (up to 32 waves/CU).  Measures fused, AES-only, HMAC-only, and
// AES(chunk i+1) || HMAC(chunk i) on two streams; checks bit-exactness.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build_tools/split_probe tools/split_probe.hip \
//         reticulum_amd/csrc/token_kernels.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../reticulum_amd/csrc/token_device.h"
#include "../reticulum_amd/csrc/token_launch.h"

using namespace rnstok;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <bool DEC>
__device__ void fill(uint32_t *tab, const uint8_t *sbox) {
    for (uint32_t d = threadIdx.x; d < 32768u; d += blockDim.x) {
        uint32_t x = (d >> 6) & 255u, t = ((d >> 14) << 1) | ((d >> 5) & 1u);
        uint32_t s = sbox[x], s2 = ((s << 1) ^ ((s & 0x80u) ? 0x1bu : 0u)) & 0xffu;
        uint32_t v = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
        tab[d] = t ? ((v << (8 * t)) | (v >> (32 - 8 * t))) : v;
    }
    __syncthreads();
}

// AES-256-CBC over uniform 500-B packets, writes iv || ct (no MAC).
__global__ __launch_bounds__(1024) void k_aes_only(const uint32_t *rec, const uint8_t *sbox, const uint8_t *pt,
                                                   uint32_t L, const uint8_t *ivs, uint8_t *tok, uint32_t tl,
                                                   uint32_t n0, uint32_t n1) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    fill<false>(tab, sbox);
    const Lanes LN(threadIdx.x & 31u);
    uint32_t rk[60];
    for (int i = 0; i < 60; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rec[i]);
    Sha256 S;
    for (uint32_t p = n0 + blockIdx.x * blockDim.x + threadIdx.x; p < n1; p += gridDim.x * blockDim.x) {
        const uint8_t *P = pt + (uint64_t)p * L;
        uint8_t *C = tok + (uint64_t)p * tl;
        u32x4 prev = ld16(ivs + 16ull * p);
        st16(C, prev);
        C += 16;
        const uint32_t nfull = L >> 4, nq = nfull >> 2, tb = (nfull & 3u) + 1u;
        u32x4 x[4], c[4];
        for (uint32_t q = 0; q < nq; ++q) {
            x[0] = ld16(P); x[1] = ld16(P + 16); x[2] = ld16(P + 32); x[3] = ld16(P + 48);
            enc_quad<14, false>(c, x, prev, rk, LN, S);
            st16(C, c[0]); st16(C + 16, c[1]); st16(C + 32, c[2]); st16(C + 48, c[3]);
            prev = c[3];
            P += 64; C += 64;
        }
        const u32x4 z = {0u, 0u, 0u, 0u};
        const uint32_t r = L & 15u;
        for (int j = 0; j < 4; ++j) {
            if ((uint32_t)j + 1u < tb) x[j] = ld16(P + 16 * j);
            else if ((uint32_t)j + 1u == tb) {
                uint32_t nn = 16u - r, w[4] = {0, 0, 0, 0};
                for (int i = 0; i < 16; ++i) w[i >> 2] |= ((uint32_t)i < r ? (uint32_t)P[16 * j + i] : nn) << (8 * (i & 3));
                x[j] = u32x4{w[0], w[1], w[2], w[3]};
            } else x[j] = z;
        }
        enc_quad<14, false>(c, x, prev, rk, LN, S);
        for (uint32_t j = 0; j < tb; ++j) st16(C + 16 * j, c[j]);
    }
}

// HMAC-SHA256 over iv || ct of uniform tokens, writes the tag.  No LDS.
__global__ __launch_bounds__(256) void k_hmac_only(const uint32_t *rec, uint8_t *tok, uint32_t tl, uint32_t n0,
                                                   uint32_t n1) {
    for (uint32_t p = n0 + blockIdx.x * blockDim.x + threadIdx.x; p < n1; p += gridDim.x * blockDim.x) {
        uint8_t *T = tok + (uint64_t)p * tl;
        const uint32_t M = tl - 32;               // iv || ct
        uint32_t h[8], opad[8];
        for (int i = 0; i < 8; ++i) { h[i] = rec[REC_IPAD + i]; opad[i] = rec[REC_OPAD + i]; }
        uint32_t full = M / 64, i = 0;
        for (; i < full; ++i) {
            uint32_t w[16];
            sha_units(w, ld16(T + 64 * i), ld16(T + 64 * i + 16), ld16(T + 64 * i + 32), ld16(T + 64 * i + 48));
            sha256_compress(h, w);
        }
        const uint32_t fu = (M - 64 * full) / 16;   // 0..3 units left
        const u32x4 z = {0u, 0u, 0u, 0u};
        const uint8_t *R = T + 64 * full;
        sha_final_units(h, fu, fu > 0 ? ld16(R) : z, fu > 1 ? ld16(R + 16) : z, fu > 2 ? ld16(R + 32) : z,
                        (uint64_t)(64 + M) * 8);
        uint32_t tag[8];
        hmac_outer(tag, h, opad);
        st16(T + M, u32x4{bswap(tag[0]), bswap(tag[1]), bswap(tag[2]), bswap(tag[3])});
        st16(T + M + 16, u32x4{bswap(tag[4]), bswap(tag[5]), bswap(tag[6]), bswap(tag[7])});
    }
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    CHECK(configure_kernels());
    CHECK(hipFuncSetAttribute((const void *)k_aes_only, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    const uint32_t n = 1u << 20, L = 500, tl = 560;
    // S-box
    uint8_t sb[512];
    {
        uint8_t ex[256], lg[256], x = 1;
        for (int i = 0; i < 255; ++i) { ex[i] = x; lg[x] = (uint8_t)i; x = (uint8_t)(x ^ (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0))); }
        for (int v = 0; v < 256; ++v) {
            uint8_t b = v ? ex[(255 - lg[v]) % 255] : 0, r = b;
            for (int i = 0; i < 4; ++i) { b = (uint8_t)((b << 1) | (b >> 7)); r ^= b; }
            r ^= 0x63; sb[v] = r; sb[256 + r] = (uint8_t)v;
        }
    }
    std::vector<uint8_t> hpt((size_t)n * L), hiv((size_t)n * 16), key(64);
    srand(1);
    for (auto &b : hpt) b = rand() & 255;
    for (auto &b : hiv) b = rand() & 255;
    for (auto &b : key) b = rand() & 255;
    uint8_t *dsb, *dpt, *div, *dtok1, *dtok2, *dkey;
    uint32_t *rec;
    CHECK(hipMalloc(&dsb, 512)); CHECK(hipMalloc(&dpt, hpt.size())); CHECK(hipMalloc(&div, hiv.size()));
    CHECK(hipMalloc(&dtok1, (size_t)n * tl)); CHECK(hipMalloc(&dtok2, (size_t)n * tl)); CHECK(hipMalloc(&dkey, 64));
    CHECK(hipMalloc(&rec, REC_WORDS * 4));
    CHECK(hipMemcpy(dsb, sb, 512, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dpt, hpt.data(), hpt.size(), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(div, hiv.data(), hiv.size(), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dkey, key.data(), 64, hipMemcpyHostToDevice));
    CHECK(launch_key_setup(dkey, 64, 1, dsb, rec, 0));
    EncArgs a{};
    a.rec = rec; a.sbox = dsb; a.pt = dpt; a.pt_stride = L; a.uni_len = L; a.iv = div; a.tok = dtok1;
    a.tok_stride = tl; a.n = n;
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto fn) {
        fn(); CHECK(hipDeviceSynchronize());
        float best = 1e9f;
        for (int r = 0; r < 7; ++r) {
            CHECK(hipEventRecord(e0, 0));
            fn();
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            CHECK(hipDeviceSynchronize());
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-44s %.4f ms  (%.3f Gpkt/s)\n", name, best, n / best / 1e6);
    };
    timeit("fused k_encrypt", [&] { CHECK(launch_encrypt(a, 14, ncu, nullptr, 0)); });
    timeit("AES-only (1024 thr x CUs)", [&] {
        hipLaunchKernelGGL(k_aes_only, dim3(ncu), dim3(1024), 131072, 0, rec, dsb, dpt, L, div, dtok2, tl, 0, n);
    });
    for (int thr : {256}) {
        timeit("HMAC-only (256 thr, 8 WG/CU)", [&] {
            hipLaunchKernelGGL(k_hmac_only, dim3(ncu * 8), dim3(thr), 0, 0, rec, dtok2, tl, 0, n);
        });
    }
    // check: AES-only + HMAC-only == fused
    {
        std::vector<uint8_t> t1((size_t)n * tl), t2((size_t)n * tl);
        CHECK(hipMemcpy(t1.data(), dtok1, t1.size(), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(t2.data(), dtok2, t2.size(), hipMemcpyDeviceToHost));
        printf("split == fused: %s\n", memcmp(t1.data(), t2.data(), t1.size()) == 0 ? "yes" : "NO");
    }
    // concurrent: chunks; AES(i+1) on s1 || HMAC(i) on s2
    for (int chunks : {4, 8, 16}) {
        char name[64];
        snprintf(name, sizeof name, "concurrent AES||HMAC, %d chunks", chunks);
        std::vector<hipEvent_t> done(chunks);
        for (auto &ev : done) CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        timeit(name, [&] {
            CHECK(hipEventRecord(e0, 0));
            CHECK(hipStreamWaitEvent(s1, e0, 0));
            CHECK(hipStreamWaitEvent(s2, e0, 0));
            const uint32_t per = n / chunks;
            for (int c = 0; c < chunks; ++c) {
                hipLaunchKernelGGL(k_aes_only, dim3(ncu), dim3(1024), 131072, s1, rec, dsb, dpt, L, div, dtok2, tl,
                                   c * per, (c + 1) * per);
                CHECK(hipEventRecord(done[c], s1));
                CHECK(hipStreamWaitEvent(s2, done[c], 0));
                hipLaunchKernelGGL(k_hmac_only, dim3(ncu * 4), dim3(256), 0, s2, rec, dtok2, tl, c * per, (c + 1) * per);
            }
            CHECK(hipEventRecord(e1, s2));
            CHECK(hipStreamWaitEvent(0, e1, 0));
        });
        std::vector<uint8_t> t1((size_t)n * tl), t2((size_t)n * tl);
        CHECK(hipMemcpy(t1.data(), dtok1, t1.size(), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(t2.data(), dtok2, t2.size(), hipMemcpyDeviceToHost));
        printf("  concurrent == fused: %s\n", memcmp(t1.data(), t2.data(), t1.size()) == 0 ? "yes" : "NO");
    }
    return 0;
}
