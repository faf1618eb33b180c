// keysetup_device.h — per-key record construction (Token.__init__,
// RNS/Cryptography/Token.py:58-74, plus the per-call work the reference
// repeats on every encrypt/decrypt: the AES key schedule aes256.py:146-175 /
// aes128.py and the HMAC key pad HMAC.py:73-82).
//
// Shared by k_key_setup (raw keys from memory, token_kernels.hip) and
// k_hkdf_key_setup (keys derived in registers, hkdf_kernels.hip).
#pragma once
#include "token_device.h"

namespace rnstok {

// Packed GF(2^8) doubling of the four bytes of a word (xtime, aes256.py:86).
__device__ __forceinline__ uint32_t xt4(uint32_t x) {
    return ((x & 0x7f7f7f7fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1bu);
}
// InvMixColumns of one column (aes256.py:101 inv_mix_columns): byte i of the
// result is 14*a_i ^ 11*a_{i+1} ^ 13*a_{i+2} ^ 9*a_{i+3}.
__device__ __forceinline__ uint32_t inv_mix_word(uint32_t x) {
    const uint32_t x2 = xt4(x), x4 = xt4(x2), x8 = xt4(x4);
    return (x8 ^ x4 ^ x2) ^ rotr(x8 ^ x2 ^ x, 8) ^ rotr(x8 ^ x4 ^ x, 16) ^ rotr(x8 ^ x, 24);
}
__device__ __forceinline__ uint32_t sub_word(const uint8_t *sb, uint32_t w) {
    return (uint32_t)sb[w & 255u] | ((uint32_t)sb[(w >> 8) & 255u] << 8) | ((uint32_t)sb[(w >> 16) & 255u] << 16) |
           ((uint32_t)sb[w >> 24] << 24);
}

// Records are written through LDS.  A lane's record is 34 16-B pieces at a
// 544-B lane stride, so a direct store instruction would touch 64 lines; each
// wave stages KS_P pieces of its 64 records per round and stores them as runs
// of KS_P * 16 contiguous bytes.  Records of consecutive keys are adjacent.
#ifndef RNSTOK_KS_P
#define RNSTOK_KS_P 12
#endif
constexpr int KS_P = RNSTOK_KS_P, KS_PIECES = REC_WORDS / 4, KS_ROUNDS = (KS_PIECES + KS_P - 1) / KS_P;
constexpr int KS_STAGE_PIECES = 64 * KS_P;     // per wave

// Lanes of one wave exchange data through LDS: order the wave's LDS writes
// before the other lanes' reads (no workgroup barrier: each wave stages only
// its own records).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Build and store the records of keys kbase .. kbase+63 (one per lane; lanes
// past n_keys compute a copy of the last key and store nothing).
//   ekw: the AES key (key[HALF:]) as NK little-endian words
//   skw: the HMAC key (key[:HALF]) as 16 big-endian words, zero padded
//   sb:  the S-box in LDS;  st: this wave's KS_STAGE_PIECES staging pieces
template <int NK>
__device__ __forceinline__ void key_record(const uint8_t *sb, const uint32_t ekw[NK], const uint32_t skw[16],
                                          u32x4 *st, uint32_t lane, uint32_t kbase, uint32_t n_keys,
                                          uint32_t *rec_out) {
    constexpr int NR = NK + 6, TOTAL = 4 * (NR + 1);
    // HMAC midstates first, so the 4*(NR+1) schedule words are not live
    // across the two compressions (k_hkdf_key_setup stays at 3 waves/SIMD).
    // HMAC midstates (HMAC.py:73-82): sk zero-padded to 64 B, ^0x36 / ^0x5c
    uint32_t bi[16], bo[16], hi[8], ho[8];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        bi[i] = skw[i] ^ 0x36363636u;
        bo[i] = skw[i] ^ 0x5c5c5c5cu;
    }
    const uint32_t iv0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
#pragma unroll
    for (int i = 0; i < 8; ++i) hi[i] = ho[i] = iv0[i];
    sha256_compress_fenced(hi, bi);
    sha256_compress_fenced(ho, bo);
    uint32_t w[TOTAL];
#pragma unroll
    for (int i = 0; i < NK; ++i) w[i] = ekw[i];
    uint32_t rcon = 1;
#pragma unroll
    for (int i = NK; i < TOTAL; ++i) {          // aes256.py:146-175 (aes128.py for NK = 4)
        uint32_t t = w[i - 1];
        if (i % NK == 0) {
            t = sub_word(sb, (t >> 8) | (t << 24)) ^ rcon;      // RotWord, SubWord, Rcon in byte 0
            rcon = xt4(rcon);
        } else if (NK > 6 && i % NK == 4) {
            t = sub_word(sb, t);
        }
        w[i] = w[i - NK] ^ t;
    }
    u32x4 *out = (u32x4 *)rec_out;
    const uint32_t nvalid = kbase < n_keys ? (n_keys - kbase < 64u ? n_keys - kbase : 64u) : 0u;
#pragma unroll
    for (int r = 0; r < KS_ROUNDS; ++r) {
#pragma unroll
        for (int j = 0; j < KS_P; ++j) {
            const int c = r * KS_P + j;              // piece c of the record: words 4c..4c+3
            if (c < KS_PIECES) {
                u32x4 d = {0u, 0u, 0u, 0u};
                if (c < 15) {                        // REC_ENC: round keys
                    if (4 * c < TOTAL) d = u32x4{w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]};
                } else if (c < 30) {                 // REC_DEC: dk[0] = rk[nr], dk[q] = InvMix(rk[nr-q]), dk[nr] = rk[0]
                    const int q = c - 15;
                    if (q <= NR) {
                        const int o = 4 * (NR - q);
                        d = (q == 0 || q == NR) ? u32x4{w[o], w[o + 1], w[o + 2], w[o + 3]}
                                                : u32x4{inv_mix_word(w[o]), inv_mix_word(w[o + 1]),
                                                        inv_mix_word(w[o + 2]), inv_mix_word(w[o + 3])};
                    }
                } else if (c == 30) {
                    d = u32x4{hi[0], hi[1], hi[2], hi[3]};
                } else if (c == 31) {
                    d = u32x4{hi[4], hi[5], hi[6], hi[7]};
                } else if (c == 32) {
                    d = u32x4{ho[0], ho[1], ho[2], ho[3]};
                } else {
                    d = u32x4{ho[4], ho[5], ho[6], ho[7]};
                }
                st[lane * KS_P + j] = d;
            }
        }
        wave_lds_sync();
        const uint32_t NP = (KS_PIECES - r * KS_P) < KS_P ? (KS_PIECES - r * KS_P) : KS_P;   // constant once unrolled
        for (uint32_t t = lane; t < nvalid * NP; t += 64u) {
            const uint32_t rr = t / NP, pc = t - rr * NP;
            out[(uint64_t)(kbase + rr) * KS_PIECES + r * KS_P + pc] = st[rr * KS_P + pc];
        }
        wave_lds_sync();
    }
}

}  // namespace rnstok
