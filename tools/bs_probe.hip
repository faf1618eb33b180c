// bs_probe.hip — would a bitsliced AES-256-CBC (pure VALU, no LDS tables)
// beat the T-table chain on gfx950?  Encrypts n packets x nblk blocks (CBC,
// no pad, no MAC) with the layout of tools/bs_aes.h: lane (g, c) of a wave
// holds column c of 32 packets as 32 bit planes, a wave covers 512 packets.
// Checks a sample against a scalar host AES-CBC; prints kernel ms.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build_tools/bs_probe tools/bs_probe.hip
//   build_tools/bs_probe [n] [nblk]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "bs_aes.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

#ifndef BS_WG
#define BS_WG 256
#endif

// ShiftRows: row r of column c comes from column (c + r) & 3 = lane (c + r) & 3 of the quad.
__device__ __forceinline__ uint32_t qperm(uint32_t v, int r) {
    if (r == 1) return __builtin_amdgcn_update_dpp(0, (int)v, 0x39, 0xF, 0xF, false);
    if (r == 2) return __builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    return __builtin_amdgcn_update_dpp(0, (int)v, 0x93, 0xF, 0xF, false);
}

template <int MODE>   // 0: full (loads + stores), 1: no memory in the block loop (compute only)
__global__ __launch_bounds__(BS_WG) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_bs_cbc(
    const uint32_t *rk_bs, const uint8_t *pt, const uint8_t *iv, uint8_t *ct, uint32_t n, uint32_t nblk,
    uint32_t stride, uint32_t ct_stride) {
    __shared__ uint32_t srk[15 * 4 * 32];
    for (uint32_t i = threadIdx.x; i < 15 * 4 * 32; i += blockDim.x) srk[i] = rk_bs[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, g = lane >> 2;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = gridDim.x * blockDim.x / 64u;
    for (uint32_t wbase = wave * 512u; wbase < n; wbase += nwaves * 512u) {
        const uint32_t p0 = wbase + g * 32u;
        uint32_t ch[32];
#pragma unroll
        for (int j = 0; j < 32; ++j)
            ch[j] = p0 + j < n ? *(const uint32_t *)(iv + 16ull * (p0 + j) + 4 * c) : 0u;
        bs_transpose(ch);
        for (uint32_t b = 0; b < nblk; ++b) {
            uint32_t s[32];
            if (MODE == 0) {
#pragma unroll
                for (int j = 0; j < 32; ++j)
                    s[j] = p0 + j < n ? *(const uint32_t *)(pt + (uint64_t)(p0 + j) * stride + 16 * b + 4 * c) : 0u;
                bs_transpose(s);
            } else {
#pragma unroll
                for (int j = 0; j < 32; ++j) s[j] = ch[j] * 0x9e3779b9u + b;
            }
            const uint32_t *k0 = srk + c * 32;
#pragma unroll
            for (int q = 0; q < 32; ++q) s[q] ^= ch[q] ^ k0[q];
#pragma unroll 1
            for (int r = 1; r <= 14; ++r) {
#pragma unroll
                for (int row = 1; row < 4; ++row)
#pragma unroll
                    for (int k = 0; k < 8; ++k) s[8 * row + k] = qperm(s[8 * row + k], row);
#pragma unroll
                for (int row = 0; row < 4; ++row) bs_sbox(s + 8 * row);
                const uint32_t *kr = srk + (r * 4 + c) * 32;
                if (r < 14) {
                    bs_mix_ark((uint32_t(*)[8])s, kr);
                } else {
#pragma unroll
                    for (int q = 0; q < 32; ++q) s[q] ^= kr[q];
                }
            }
#pragma unroll
            for (int q = 0; q < 32; ++q) ch[q] = s[q];
            if (MODE == 0) {
                bs_transpose(s);
#pragma unroll
                for (int j = 0; j < 32; ++j)
                    if (p0 + j < n) *(uint32_t *)(ct + (uint64_t)(p0 + j) * ct_stride + 16 * b + 4 * c) = s[j];
            }
        }
        if (MODE == 1) {   // keep the result live
            uint32_t x = 0;
#pragma unroll
            for (int q = 0; q < 32; ++q) x ^= ch[q];
            if (x == 0x12345678u) ct[lane] = 1;
        }
    }
}

// ---- host scalar AES-256 (FIPS-197) for the check ----
static uint8_t SB[256];
static uint8_t xt(uint8_t b) { return (uint8_t)((b << 1) ^ ((b & 0x80) ? 0x1b : 0)); }
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) { if (b & 1) p ^= a; a = xt(a); b >>= 1; }
    return p;
}
static void make_sbox() {
    for (int v = 0; v < 256; ++v) {
        uint8_t inv = 0;
        for (int y = 1; y < 256 && v; ++y) if (gmul((uint8_t)v, (uint8_t)y) == 1) inv = (uint8_t)y;
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; ++i) { r = (uint8_t)((r << 1) | (r >> 7)); s ^= r; }
        SB[v] = s ^ 0x63;
    }
}
static void expand(const uint8_t key[32], uint32_t w[60]) {
    for (int i = 0; i < 8; ++i) w[i] = key[4 * i] | key[4 * i + 1] << 8 | key[4 * i + 2] << 16 | (uint32_t)key[4 * i + 3] << 24;
    uint8_t rc = 1;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = w[i - 1];
        if (i % 8 == 0) {
            t = (t >> 8) | (t << 24);
            t = SB[t & 255] | SB[(t >> 8) & 255] << 8 | SB[(t >> 16) & 255] << 16 | (uint32_t)SB[t >> 24] << 24;
            t ^= rc; rc = xt(rc);
        } else if (i % 8 == 4) {
            t = SB[t & 255] | SB[(t >> 8) & 255] << 8 | SB[(t >> 16) & 255] << 16 | (uint32_t)SB[t >> 24] << 24;
        }
        w[i] = w[i - 8] ^ t;
    }
}
static void enc_block(const uint32_t w[60], uint8_t s[16]) {
    for (int i = 0; i < 16; ++i) s[i] ^= (uint8_t)(w[i / 4] >> (8 * (i % 4)));
    for (int r = 1; r <= 14; ++r) {
        uint8_t t[16];
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row) t[4 * c + row] = SB[s[4 * ((c + row) & 3) + row]];
        if (r < 14)
            for (int c = 0; c < 4; ++c) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3], x = a0 ^ a1 ^ a2 ^ a3;
                t[4 * c] ^= x ^ xt(a0 ^ a1); t[4 * c + 1] ^= x ^ xt(a1 ^ a2);
                t[4 * c + 2] ^= x ^ xt(a2 ^ a3); t[4 * c + 3] ^= x ^ xt(a3 ^ a0);
            }
        for (int i = 0; i < 16; ++i) s[i] = t[i] ^ (uint8_t)(w[4 * r + i / 4] >> (8 * (i % 4)));
    }
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : (1u << 20), nblk = argc > 2 ? atoi(argv[2]) : 32;
    const uint32_t stride = 16 * nblk;
    make_sbox();
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(7 * i + 1);
    uint32_t w[60];
    expand(key, w);
    std::vector<uint32_t> rkbs(15 * 4 * 32);
    for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 4; ++c)
            for (int q = 0; q < 32; ++q) rkbs[(r * 4 + c) * 32 + q] = ((w[4 * r + c] >> q) & 1) ? 0xffffffffu : 0u;
    std::vector<uint8_t> hpt((size_t)n * stride), hiv((size_t)n * 16);
    uint64_t x = 88172645463325252ull;
    for (auto &v : hpt) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint8_t)x; }
    for (auto &v : hiv) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint8_t)x; }
    uint32_t *drk; uint8_t *dpt, *div, *dct;
    CHECK(hipMalloc(&drk, rkbs.size() * 4));
    CHECK(hipMalloc(&dpt, hpt.size()));
    CHECK(hipMalloc(&div, hiv.size()));
    CHECK(hipMalloc(&dct, hpt.size()));
    CHECK(hipMemcpy(drk, rkbs.data(), rkbs.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dpt, hpt.data(), hpt.size(), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(div, hiv.data(), hiv.size(), hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const uint32_t waves = (n + 511) / 512, wpb = BS_WG / 64;
    uint32_t grid = (waves + wpb - 1) / wpb;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int mode = 0; mode < 2; ++mode) {
        std::vector<float> ms;
        for (int it = 0; it < 12; ++it) {
            CHECK(hipEventRecord(e0, 0));
            if (mode == 0) hipLaunchKernelGGL(k_bs_cbc<0>, dim3(grid), dim3(BS_WG), 0, 0, drk, dpt, div, dct, n, nblk, stride, stride);
            else hipLaunchKernelGGL(k_bs_cbc<1>, dim3(grid), dim3(BS_WG), 0, 0, drk, dpt, div, dct, n, nblk, stride, stride);
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float t; CHECK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 2) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("%s: n=%u nblk=%u grid=%u x %d: median %.4f ms  min %.4f ms  (%.1f G blocks/s)\n",
               mode == 0 ? "bitsliced CBC (loads+stores)" : "bitsliced CBC (compute only)", n, nblk, grid, BS_WG,
               ms[ms.size() / 2], ms[0], (double)n * nblk / (ms[ms.size() / 2] * 1e-3) / 1e9);
        if (mode == 0) {
            std::vector<uint8_t> hct(hpt.size());
            CHECK(hipMemcpy(hct.data(), dct, hct.size(), hipMemcpyDeviceToHost));
            int bad = 0;
            for (uint32_t p = 0; p < n && bad < 5; p += (p < 2048 ? 1 : 997)) {
                uint8_t prev[16];
                memcpy(prev, &hiv[16ull * p], 16);
                for (uint32_t b = 0; b < nblk; ++b) {
                    uint8_t s[16];
                    for (int i = 0; i < 16; ++i) s[i] = hpt[(size_t)p * stride + 16 * b + i] ^ prev[i];
                    enc_block(w, s);
                    if (memcmp(s, &hct[(size_t)p * stride + 16 * b], 16)) { printf("MISMATCH packet %u block %u\n", p, b); ++bad; break; }
                    memcpy(prev, s, 16);
                }
            }
            printf("check: %s\n", bad ? "FAIL" : "bit-exact vs host AES-256-CBC");
            if (bad) return 1;
        }
    }
    return 0;
}
