// token_device.h — CDNA4 device primitives for the encrypted-token kernels.
//
// AES (FIPS-197) as T-table rounds over LDS, SHA-256 (FIPS 180-4) in VGPRs.
// Reference semantics: RNS/Cryptography/aes/aes256.py:177-235 (block cipher,
// CBC), RNS/Cryptography/HMAC.py:47-125 (HMAC), Token.py:87-114 (token).
//
// LDS table image (one workgroup per CU owns it):
//   region 0 [0x00000,0x10000): 256 rows x 256 B; dwords 0-31 = T0[x], 32-63 = T1[x]
//   region 1 [0x10000,0x20000): same rows for T2[x] / T3[x]
//   region 2 [0x20000,0x28000): (decrypt only) 256 rows x 128 B of InvS[x]*0x01010101
// Every table entry is replicated 32 times across the 32 banks a ds_read_b32
// lane-group sees, so lane l always reads bank (l & 31): conflict-free for
// any data.  The LDS byte address of a lookup is built by ONE v_perm_b32:
//   addr = { lane_off(8b), state byte x (8b), region (8b), 0 }
// and the table (T0 vs T1, T2 vs T3) is selected by the ds_read immediate
// offset (0 or 128).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnstok {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Key record (u32 words), produced by k_key_setup:
constexpr int REC_WORDS = 136;          // 544 B, 16-B aligned
constexpr int REC_ENC = 0;              // 4*(Nr+1) words of encryption round keys
constexpr int REC_DEC = 60;             // equivalent-inverse-cipher round keys
constexpr int REC_IPAD = 120;           // SHA-256 state after (sk ^ ipad)
constexpr int REC_OPAD = 128;           // SHA-256 state after (sk ^ opad)

constexpr uint32_t LDS_ENC_BYTES = 0x20000;   // 128 KiB
constexpr uint32_t LDS_DEC_BYTES = 0x28000;   // 160 KiB

// v_perm_b32 selectors: byte i of the result picks byte sel_i of {S0:S1}
// (0-3 = S1 bytes, 4-7 = S0 bytes, 0x0c = 0x00).
// S0 = state word, S1 = lane constant {lane_off, -, region, 0}.
template <int K> struct Sel {
    static constexpr uint32_t R0 = 0x0C0C0000u | ((4u + K) << 8);   // region 0
    static constexpr uint32_t R1 = 0x0C020000u | ((4u + K) << 8);   // region from lane const byte 2
};

__device__ __forceinline__ uint32_t perm(uint32_t s, uint32_t lc, uint32_t sel) {
    return __builtin_amdgcn_perm(s, lc, sel);
}

// LDS read at an absolute byte address of the workgroup's LDS (the table
// image is the only LDS allocation and starts at 0, see fill_tables), so the
// v_perm_b32 result is the ds_read address with no base add.
typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds(const char *, uint32_t addr, uint32_t off) {
    return *(lds_u32_t *)(uintptr_t)(addr + off);
}

// v_bitop3_b32 (gfx950): any 3-input bitwise function in one VALU op.
// 0x96 = a ^ b ^ c, 0xE8 = majority(a, b, c) (both symmetric in a, b, c).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) { __builtin_memcpy(p, &v, 16); }

__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
    return (a & mask) | (b & ~mask);
}

// ------------------------------------------------------------------ AES --

// One encryption round: t_j = T0[s_j.b0] ^ T1[s_{j+1}.b1] ^ T2[s_{j+2}.b2] ^ T3[s_{j+3}.b3] ^ rk_j
#define RT_ENC_COL(o, a, b, c, d, k)                                                        \
    o = xor3(xor3(lds(tab, perm(a, lc, Sel<0>::R0), 0), lds(tab, perm(b, lc, Sel<1>::R0), 128),  \
                  lds(tab, perm(c, lc, Sel<2>::R1), 0)),                                     \
             lds(tab, perm(d, lc, Sel<3>::R1), 128), (k))

// Final round: row r taken from the table whose byte r is S[x]:
// row0 <- T2 (region1,+0), row1 <- T3 (region1,+128), row2 <- T0 (region0,+0), row3 <- T1 (region0,+128)
#define RT_ENC_LAST(o, a, b, c, d, k)                                                       \
    o = bfi(0x000000ffu, lds(tab, perm(a, lc, Sel<0>::R1), 0),                              \
        bfi(0x0000ff00u, lds(tab, perm(b, lc, Sel<1>::R1), 128),                            \
        bfi(0x00ff0000u, lds(tab, perm(c, lc, Sel<2>::R0), 0),                              \
                          lds(tab, perm(d, lc, Sel<3>::R0), 128)))) ^ (k)

// x = plaintext ^ chaining value (caller); rk = NR+1 round keys.
template <int NR>
__device__ __forceinline__ u32x4 aes_enc(u32x4 x, const uint32_t *rk, uint32_t lc, const char *tab) {
    uint32_t s0 = x.x ^ rk[0], s1 = x.y ^ rk[1], s2 = x.z ^ rk[2], s3 = x.w ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        uint32_t t0, t1, t2, t3;
        RT_ENC_COL(t0, s0, s1, s2, s3, rk[4 * r + 0]);
        RT_ENC_COL(t1, s1, s2, s3, s0, rk[4 * r + 1]);
        RT_ENC_COL(t2, s2, s3, s0, s1, rk[4 * r + 2]);
        RT_ENC_COL(t3, s3, s0, s1, s2, rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    u32x4 o;
    RT_ENC_LAST(o.x, s0, s1, s2, s3, rk[4 * NR + 0]);
    RT_ENC_LAST(o.y, s1, s2, s3, s0, rk[4 * NR + 1]);
    RT_ENC_LAST(o.z, s2, s3, s0, s1, rk[4 * NR + 2]);
    RT_ENC_LAST(o.w, s3, s0, s1, s2, rk[4 * NR + 3]);
    return o;
}

// Decryption round (equivalent inverse cipher):
// t_j = Td0[s_j.b0] ^ Td1[s_{j-1}.b1] ^ Td2[s_{j-2}.b2] ^ Td3[s_{j-3}.b3] ^ dk_j
// Final: InvS bytes from region 2 (row stride 128 B): addr = perm(s, lc2, R1) >> 1,
// with lc2 = {8*(lane&31), -, 4, 0}.
#define RT_DEC_INV(a, k) (lds(tab, perm(a, lc2, Sel<k>::R1) >> 1, 0))
#define RT_DEC_LAST(o, a, b, c, d, kk)                                                      \
    o = bfi(0x000000ffu, RT_DEC_INV(a, 0),                                                  \
        bfi(0x0000ff00u, RT_DEC_INV(b, 1),                                                  \
        bfi(0x00ff0000u, RT_DEC_INV(c, 2), RT_DEC_INV(d, 3)))) ^ (kk)

template <int NR>
__device__ __forceinline__ u32x4 aes_dec(u32x4 x, const uint32_t *dk, uint32_t lc, uint32_t lc2,
                                         const char *tab) {
    uint32_t s0 = x.x ^ dk[0], s1 = x.y ^ dk[1], s2 = x.z ^ dk[2], s3 = x.w ^ dk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        uint32_t t0, t1, t2, t3;
        RT_ENC_COL(t0, s0, s3, s2, s1, dk[4 * r + 0]);
        RT_ENC_COL(t1, s1, s0, s3, s2, dk[4 * r + 1]);
        RT_ENC_COL(t2, s2, s1, s0, s3, dk[4 * r + 2]);
        RT_ENC_COL(t3, s3, s2, s1, s0, dk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    u32x4 o;
    RT_DEC_LAST(o.x, s0, s3, s2, s1, dk[4 * NR + 0]);
    RT_DEC_LAST(o.y, s1, s0, s3, s2, dk[4 * NR + 1]);
    RT_DEC_LAST(o.z, s2, s1, s0, s3, dk[4 * NR + 2]);
    RT_DEC_LAST(o.w, s3, s2, s1, s0, dk[4 * NR + 3]);
    return o;
}

// -------------------------------------------------------------- SHA-256 --

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void sha256_compress(uint32_t h[8], uint32_t w[16]) {
    constexpr uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] = (w[i & 15] + s0 + w[(i + 9) & 15]) + s1;
        }
        const uint32_t t1 = (hh + K[i] + wi) + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + bfi(e, f, g);
        const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj3(a, b, c);
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// SHA-256 message words from four 16-B units (big-endian words).
__device__ __forceinline__ void sha_units(uint32_t w[16], u32x4 a, u32x4 b, u32x4 c, u32x4 d) {
    w[0] = bswap(a.x); w[1] = bswap(a.y); w[2] = bswap(a.z); w[3] = bswap(a.w);
    w[4] = bswap(b.x); w[5] = bswap(b.y); w[6] = bswap(b.z); w[7] = bswap(b.w);
    w[8] = bswap(c.x); w[9] = bswap(c.y); w[10] = bswap(c.z); w[11] = bswap(c.w);
    w[12] = bswap(d.x); w[13] = bswap(d.y); w[14] = bswap(d.z); w[15] = bswap(d.w);
}

// Final padded SHA block holding fu (0..3) 16-B units s0..s2 of the message,
// then 0x80, zeros and the 64-bit big-endian bit length.
__device__ __forceinline__ void sha_final_units(uint32_t h[8], uint32_t fu, u32x4 s0, u32x4 s1, u32x4 s2,
                                                uint64_t bits) {
    uint32_t w[16];
    const u32x4 z = {0u, 0u, 0u, 0u};
    sha_units(w, fu > 0 ? s0 : z, fu > 1 ? s1 : z, fu > 2 ? s2 : z, z);
#pragma unroll
    for (int k = 0; k < 16; k += 4) {
        uint32_t hit = (uint32_t)(4 * fu) == (uint32_t)k ? 0x80000000u : 0u;
        w[k] |= hit;
    }
    w[14] = (uint32_t)(bits >> 32);
    w[15] |= (uint32_t)bits;
    sha256_compress(h, w);
}

// HMAC outer hash: tag = SHA256(opad_state, inner_digest || pad), 96-byte message.
__device__ __forceinline__ void hmac_outer(uint32_t tag[8], const uint32_t inner[8], const uint32_t opad[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) { w[i] = inner[i]; tag[i] = opad[i]; }
    w[8] = 0x80000000u;
#pragma unroll
    for (int i = 9; i < 15; ++i) w[i] = 0;
    w[15] = (64 + 32) * 8;
    sha256_compress(tag, w);
}

// Generic byte-granular HMAC inner hash (rare lanes: malformed token lengths).
// Hashes n bytes at p after the 64-byte ipad block.
__device__ __noinline__ void sha_bytes_after_ipad(uint32_t h[8], const uint8_t *p, uint64_t n) {
    uint64_t bits = (64 + n) * 8;
    uint64_t i = 0;
    uint32_t w[16];
    for (; i + 64 <= n; i += 64) {
        for (int k = 0; k < 16; ++k)
            w[k] = ((uint32_t)p[i + 4 * k] << 24) | ((uint32_t)p[i + 4 * k + 1] << 16) |
                   ((uint32_t)p[i + 4 * k + 2] << 8) | p[i + 4 * k + 3];
        sha256_compress(h, w);
    }
    uint32_t rem = (uint32_t)(n - i);
    uint8_t buf[128];
    for (uint32_t k = 0; k < 128; ++k) buf[k] = 0;
    for (uint32_t k = 0; k < rem; ++k) buf[k] = p[i + k];
    buf[rem] = 0x80;
    uint32_t blocks = rem + 9 <= 64 ? 1 : 2;
    for (int k = 0; k < 8; ++k) buf[64 * blocks - 1 - k] = (uint8_t)(bits >> (8 * k));
    for (uint32_t b = 0; b < blocks; ++b) {
        for (int k = 0; k < 16; ++k)
            w[k] = ((uint32_t)buf[64 * b + 4 * k] << 24) | ((uint32_t)buf[64 * b + 4 * k + 1] << 16) |
                   ((uint32_t)buf[64 * b + 4 * k + 2] << 8) | buf[64 * b + 4 * k + 3];
        sha256_compress(h, w);
    }
}

}  // namespace rnstok
