// l4_round_probe.hip — where the cycles of one k_encrypt_long4 AES round go
// (VERDICT r03 next #7).  The long-token encrypt (c4 per-rank shard, 128
// tokens per CU) is bound by its CBC chain: one round = 4 table addresses
// (3 v_perm + 1 v_bitop3) -> 4 ds_read_b32 -> 3 DPP quad permutes -> 2 xor3
// -> the next round's addresses.  This probe runs that round (token_device.h's
// taddr / lds and the kernel's quad_rot, same conflict-free addressing) in a
// register-resident chain and stamps one round with s_memtime:
//   t0  the round's input word is ready (readfirstlane of it)
//   t1  the four lookups have returned (s_waitcnt lgkmcnt(0) on them)
//   t2  the three DPP moves have issued
//   t3  the next input word is ready (readfirstlane of it)
// plus a calibration (two stamps back to back), at three launch shapes:
//   solo : one AES wave per CU (the chain alone: pure latency)
//   l4   : the kernel's shape, 8 AES waves + 2 hashing waves running SHA-256
//          compressions (2 AES waves on every SIMD, hashing on two of them)
//   aes8 : 8 AES waves, no hashing
// Per shape: mean cycles of each segment over the stamped rounds of wave 0 of
// every CU, and the un-stamped chain's cycles per round (wall of 4096 rounds).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build_exp/l4_round_probe tools/l4_round_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "../reticulum_amd/csrc/token_device.h"

using namespace rnstok;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int STAMPED = 32;         // rounds stamped per wave-0
constexpr int PLAIN = 4096;         // rounds of the un-stamped chain

template <int K>
__device__ __forceinline__ uint32_t quad_rot(uint32_t v) {
    constexpr int ctrl = K == 1 ? 0x39 : (K == 2 ? 0x4E : 0x93);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, true);
}

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// one round of enc_block4 (k_encrypt_long4), returns the next state word.
// Ablations (MODE): 0 the round as the kernel runs it; 1 without the DPP
// moves (the lane's own four lookups folded); 2 the LDS round trip alone
// (one address, one lookup, its result the next state); 3 without LDS (the
// "lookups" are VALU functions of the addresses), DPP and folds kept.
template <int MODE>
__device__ __forceinline__ uint32_t round4(uint32_t s, uint32_t rk, const Lanes &L) {
    if (MODE == 2) return lds(taddr<0, 0>(s, L), 0);
    uint32_t u0, u1, u2, u3;
    if (MODE == 3) {
        u0 = taddr<0, 0>(s, L) ^ 0x1234u; u1 = taddr<1, 0>(s, L) ^ 0x5678u;
        u2 = taddr<2, 1>(s, L) ^ 0x9abcu; u3 = taddr<3, 1>(s, L) ^ 0xdef0u;
        asm volatile("" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
    } else {
        u0 = lds(taddr<0, 0>(s, L), 0); u1 = lds(taddr<1, 0>(s, L), 128);
        u2 = lds(taddr<2, 1>(s, L), 0); u3 = lds(taddr<3, 1>(s, L), 128);
    }
    if (MODE == 1) return xor3(xor3(u1, u2, u3), u0, rk);
    uint32_t x1 = quad_rot<1>(u1), x2 = quad_rot<2>(u2), x3 = quad_rot<3>(u3);
    asm volatile("" : "+v"(x1), "+v"(x2), "+v"(x3));
    return xor3(xor3(x1, x2, x3), u0, rk);
}

struct Out {
    uint64_t seg[4];        // sums over stamped rounds: t1-t0, t2-t1, t3-t2, calibration
    uint64_t plain[4];      // cycles of PLAIN un-stamped rounds, per ablation MODE
    uint32_t sink;
};

template <int AES_WAVES, int HASH_WAVES>
__global__ __launch_bounds__(64 * (AES_WAVES + HASH_WAVES)) void k_probe(const uint32_t *rk_in, Out *out, uint32_t seed) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    for (uint32_t d = threadIdx.x; d < LDS_ENC_BYTES / 4; d += blockDim.x) tab[d] = d * 2654435761u + seed;
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    const Lanes L(threadIdx.x & 31u);
    uint32_t sink = 0;
    if (wave < (uint32_t)AES_WAVES) {
        const uint32_t rk = rk_in[threadIdx.x & 3u];
        uint32_t s = threadIdx.x * 0x9E3779B9u ^ seed;
        if (wave == 0) {
            uint64_t a = 0, b = 0, c = 0, cal = 0;
            for (int r = 0; r < STAMPED; ++r) {
                const uint32_t d0 = __builtin_amdgcn_readfirstlane(s);
                asm volatile("" ::"s"(d0));
                const uint64_t t0 = stamp();
                const uint32_t u0 = lds(taddr<0, 0>(s, L), 0), u1 = lds(taddr<1, 0>(s, L), 128);
                const uint32_t u2 = lds(taddr<2, 1>(s, L), 0), u3 = lds(taddr<3, 1>(s, L), 128);
                uint64_t t1;
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)"
                             : "=s"(t1) : "v"(u0), "v"(u1), "v"(u2), "v"(u3) : "memory");
                uint32_t x1 = quad_rot<1>(u1), x2 = quad_rot<2>(u2), x3 = quad_rot<3>(u3);
                asm volatile("" : "+v"(x1), "+v"(x2), "+v"(x3));
                uint64_t t2;
                asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t2) : "v"(x1), "v"(x2), "v"(x3) : "memory");
                s = xor3(xor3(x1, x2, x3), u0, rk);
                const uint32_t d3 = __builtin_amdgcn_readfirstlane(s);
                asm volatile("" ::"s"(d3));
                const uint64_t t3 = stamp();
                const uint64_t t4 = stamp();
                a += t1 - t0; b += t2 - t1; c += t3 - t2; cal += t4 - t3;
            }
            if ((threadIdx.x & 63u) == 0) {
                out[blockIdx.x].seg[0] = a; out[blockIdx.x].seg[1] = b;
                out[blockIdx.x].seg[2] = c; out[blockIdx.x].seg[3] = cal;
            }
        }
        auto chain = [&](auto mode) {
            constexpr int M = decltype(mode)::value;
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(s);
            asm volatile("" ::"s"(d0));
            const uint64_t p0 = stamp();
#pragma nounroll
            for (int r = 0; r < PLAIN; ++r) s = round4<M>(s, rk, L);
            const uint32_t d = __builtin_amdgcn_readfirstlane(s);
            asm volatile("" ::"s"(d));
            const uint64_t p1 = stamp();
            if (wave == 0 && (threadIdx.x & 63u) == 0) out[blockIdx.x].plain[M] = p1 - p0;
        };
        chain(std::integral_constant<int, 0>());
        chain(std::integral_constant<int, 1>());
        chain(std::integral_constant<int, 2>());
        chain(std::integral_constant<int, 3>());
        sink = s;
    } else {
        uint32_t h[8], w[16];
        for (int k = 0; k < 8; ++k) h[k] = seed + k + threadIdx.x;
        for (int k = 0; k < 16; ++k) w[k] = seed * 3 + k;
        // enough compressions to outlast the AES waves' chains
#pragma nounroll
        for (int i = 0; i < PLAIN / 2 + STAMPED; ++i) {
            sha256_compress(h, w);
            for (int k = 0; k < 8; ++k) w[k] ^= h[k];
        }
        sink = h[0] ^ h[7];
    }
    if (sink == 0x12345678u) out[blockIdx.x].sink = sink;
}

template <int A, int H>
static void run(const char *name, int ncu, const uint32_t *d_rk, Out *d_out) {
    auto k = k_probe<A, H>;
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ENC_BYTES));
    hipLaunchKernelGGL(k, dim3(ncu), dim3(64 * (A + H)), LDS_ENC_BYTES, 0, d_rk, d_out, 1u);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k, dim3(ncu), dim3(64 * (A + H)), LDS_ENC_BYTES, 0, d_rk, d_out, 2u);
    CHECK(hipDeviceSynchronize());
    Out *h = (Out *)malloc(sizeof(Out) * ncu);
    CHECK(hipMemcpy(h, d_out, sizeof(Out) * ncu, hipMemcpyDeviceToHost));
    double seg[4] = {0, 0, 0, 0}, plain[4] = {0, 0, 0, 0};
    for (int b = 0; b < ncu; ++b) {
        for (int i = 0; i < 4; ++i) seg[i] += (double)h[b].seg[i] / STAMPED / ncu;
        for (int i = 0; i < 4; ++i) plain[i] += (double)h[b].plain[i] / PLAIN / ncu;
    }
    printf("%-5s %2d AES + %d hash waves | stamped: lookup (addr->data) %6.1f, DPP %5.1f, xor3 -> next %5.1f, "
           "stamp alone %5.1f | chain cycles per round: full %6.1f, no DPP %6.1f, LDS round trip alone %6.1f, "
           "no LDS %6.1f\n",
           name, A, H, seg[0], seg[1], seg[2], seg[3], plain[0], plain[1], plain[2], plain[3]);
    free(h);
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    uint32_t *d_rk;
    Out *d_out;
    CHECK(hipMalloc(&d_rk, 64));
    CHECK(hipMemset(d_rk, 0x3c, 64));
    CHECK(hipMalloc(&d_out, sizeof(Out) * ncu));
    CHECK(hipMemset(d_out, 0, sizeof(Out) * ncu));
    printf("s_memtime cycles (shader clock); segments are means over %d stamped rounds of wave 0 on %d CUs\n", STAMPED,
           ncu);
    run<1, 0>("solo", ncu, d_rk, d_out);
    run<8, 0>("aes8", ncu, d_rk, d_out);
    run<8, 2>("l4", ncu, d_rk, d_out);
    return 0;
}
