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
// any data.  The LDS byte address of a lookup is
//   addr = { lane_off(8b), state byte x (8b), region (8b), 0 }
// built by one v_perm_b32 (bytes 0, 2, 3) or one v_bitop3 (byte 1, already in
// place), and the table (T0 vs T1, T2 vs T3) is selected by the ds_read
// immediate offset (0 or 128).
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
// S0 = state word, S1 = lane constant Lanes::r1 = {4*lane, -, 1, 0}.
template <int K> struct Sel {
    static constexpr uint32_t R0 = 0x0C0C0000u | ((4u + K) << 8);   // region 0
    static constexpr uint32_t R1 = 0x0C020000u | ((4u + K) << 8);   // region 1 (byte 2 of r1)
};

__device__ __forceinline__ uint32_t perm(uint32_t s, uint32_t lc, uint32_t sel) {
    return __builtin_amdgcn_perm(s, lc, sel);
}

// v_bitop3_b32 (gfx950): any 3-input bitwise function in ONE full-rate VALU op
// (measured: tools/valu_peak.hip — v_bitop3 issues at the v_add/v_xor rate
// while v_perm/v_alignbit/v_bfi/v_add3/v_and_or/SDWA issue at half rate).
// Truth table index = {S0,S1,S2} bits, i.e. TT = f(0xF0, 0xCC, 0xAA).
template <uint32_t TT>
__device__ __forceinline__ uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return bitop3<0x96>(a, b, c); }
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) { return bitop3<0xE8>(a, b, c); }
// (m & a) | (~m & b): SHA-256 Ch(e,f,g) and byte merges
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return bitop3<0xCA>(m, a, b); }
// (a & m) | c
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t c) { return bitop3<0xEA>(a, m, c); }

// LDS read at an absolute byte address of the workgroup's LDS (the table
// image is the only LDS allocation and starts at 0, see fill_tables), so the
// computed address needs no base add.
typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds(uint32_t addr, uint32_t off) {
    return *(lds_u32_t *)(uintptr_t)(addr + off);
}

__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) { __builtin_memcpy(p, &v, 16); }

// Per-lane constants for LDS addressing; lane l always hits bank (l & 31).
// A VALU op that reads an SGPR (or a constant materialised in one) issues at
// half rate on gfx950 (tools/issue_probe.hip), so the byte mask of the hot
// address computation is kept in a VGPR.
struct Lanes {
    uint32_t r0;    // 4*lane            (region 0)
    uint32_t r1;    // 4*lane | 0x10000  (region 1; also the v_perm lane constant)
    uint32_t inv;   // 4*lane | 0x20000  (region 2, InvS rows of 128 B)
    uint32_t m8;    // 0x0000ff00 in a VGPR
    __device__ __forceinline__ explicit Lanes(uint32_t lane)
        : r0(4u * lane), r1(4u * lane | 0x10000u), inv(4u * lane | 0x20000u), m8(0xff00u) {
        asm volatile("" : "+v"(m8));
    }
};

// ------------------------------------------------------------------ AES --
//
// Address of the T-table row for byte k of state word s: {lane_off, s.byte_k, region, 0}.
// Byte 1 is already in bits 8..15, so (s & 0xff00) | lane_off is one full-rate
// v_bitop3; bytes 0, 2, 3 take one (half-rate) v_perm_b32.
template <int K, int REGION, bool SHIFT = false>
__device__ __forceinline__ uint32_t taddr(uint32_t s, const Lanes &L) {
    // (Bytes 0, 2, 3 by a shift to bits 8..15 plus the same and_or, two
    // dual-issuable ops instead of one v_perm, was 7-11 % slower on c2/c3 and
    // 14 % on the c4 shard: the kernels' mixed streams do not pair them,
    // profiles/r03e_shift_addr_ab.txt.  SHIFT keeps that form for the
    // per-wave experiment of round 6.)
    if (K == 1) return and_or(s, L.m8, REGION ? L.r1 : L.r0);
    if (SHIFT) return and_or(K == 0 ? s << 8 : s >> (8 * K - 8), L.m8, REGION ? L.r1 : L.r0);
    return perm(s, L.r1, REGION ? Sel<K>::R1 : Sel<K>::R0);
}

// One T-table round column: T0[a.b0] ^ T1[b.b1] ^ T2[c.b2] ^ T3[d.b3] ^ k
// (T0/T1 in region 0 at +0/+128, T2/T3 in region 1 at +0/+128).
__device__ __forceinline__ uint32_t tcol(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k,
                                         const Lanes &L) {
    return xor3(xor3(lds(taddr<0, 0>(a, L), 0), lds(taddr<1, 0>(b, L), 128), lds(taddr<2, 1>(c, L), 0)),
                lds(taddr<3, 1>(d, L), 128), k);
}

// A round split in two so independent work can sit between the LDS reads and
// their use: tround_load issues the 16 lookups, tround_mix folds them.
// Column j reads bytes 0..3 of words (j, j+1, j+2, j+3) for encryption and
// (j, j-1, j-2, j-3) for the equivalent inverse cipher.
template <bool DEC, bool SHIFT = false>
__device__ __forceinline__ void tround_load(uint32_t v[16], const uint32_t s[4], const Lanes &L) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i1 = DEC ? (j + 3) & 3 : (j + 1) & 3, i2 = (j + 2) & 3, i3 = DEC ? (j + 1) & 3 : (j + 3) & 3;
        v[4 * j + 0] = lds(taddr<0, 0, SHIFT>(s[j], L), 0);
        v[4 * j + 1] = lds(taddr<1, 0, SHIFT>(s[i1], L), 128);
        v[4 * j + 2] = lds(taddr<2, 1, SHIFT>(s[i2], L), 0);
        v[4 * j + 3] = lds(taddr<3, 1, SHIFT>(s[i3], L), 128);
    }
}
__device__ __forceinline__ void tround_mix(uint32_t s[4], const uint32_t v[16], const uint32_t *k) {
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = xor3(xor3(v[4 * j], v[4 * j + 1], v[4 * j + 2]), v[4 * j + 3], k[j]);
}


// Encryption final round column: row r from the table whose byte r is S[x]
// (row0 <- T2, row1 <- T3, row2 <- T0, row3 <- T1), merged by byte masks.
__device__ __forceinline__ uint32_t tlast_enc(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k,
                                              const Lanes &L) {
    const uint32_t u0 = lds(taddr<0, 1>(a, L), 0), u1 = lds(taddr<1, 1>(b, L), 128);
    const uint32_t u2 = lds(taddr<2, 0>(c, L), 0), u3 = lds(taddr<3, 0>(d, L), 128);
    return bfi(0x0000ffffu, bfi(0x000000ffu, u0, u1), bfi(0x00ff0000u, u2, u3)) ^ k;
}

// Decryption final round: InvS[x] (replicated in all 4 bytes) from region 2,
// rows of 128 B: address = ((byte_k << 7) & 0x7f80) | Lanes::inv.
template <int K>
__device__ __forceinline__ uint32_t invs(uint32_t s, const Lanes &L) {
    const uint32_t t = K == 0 ? (s << 7) : (s >> (8 * K - 7));
    return lds(and_or(t, 0x7f80u, L.inv), 0);
}
__device__ __forceinline__ uint32_t tlast_dec(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k,
                                              const Lanes &L) {
    return bfi(0x0000ffffu, bfi(0x000000ffu, invs<0>(a, L), invs<1>(b, L)),
               bfi(0x00ff0000u, invs<2>(c, L), invs<3>(d, L))) ^ k;
}

// -------------------------------------------------------------- SHA-256 --

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// SHA-256 compression split into rounds so its VALU chain can be interleaved
// with an AES chain (whose time is LDS latency) inside one wave.  The eight
// working variables rotate through v[] by index instead of by moves:
// at round i, a = v[(0-i)&7], b = v[(1-i)&7], ..., h = v[(7-i)&7].
struct Sha256 {
    uint32_t v[8];
    uint32_t w[16];

    __device__ __forceinline__ void start(const uint32_t h[8]) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = h[k];
    }
    __device__ __forceinline__ void round(int i) {
        constexpr uint32_t K[64] = {
            0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
            0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
            0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
            0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
            0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
            0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
            0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
            0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] = (w[i & 15] + s0 + w[(i + 9) & 15]) + s1;
        }
        const uint32_t a = v[(0 - i) & 7], b = v[(1 - i) & 7], c = v[(2 - i) & 7], d = v[(3 - i) & 7];
        const uint32_t e = v[(4 - i) & 7], f = v[(5 - i) & 7], g = v[(6 - i) & 7], h = v[(7 - i) & 7];
        const uint32_t t1 = (h + K[i] + wi) + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + bfi(e, f, g);
        const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj3(a, b, c);
        v[(3 - i) & 7] = d + t1;      // new e
        v[(7 - i) & 7] = t1 + t2;     // new a
    }
    __device__ __forceinline__ void finish(uint32_t h[8]) {
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] += v[k];
    }
};

__device__ __forceinline__ void sha256_compress(uint32_t h[8], const uint32_t w[16]) {
    Sha256 S;
    S.start(h);
#pragma unroll
    for (int k = 0; k < 16; ++k) S.w[k] = w[k];
#pragma unroll
    for (int i = 0; i < 64; ++i) S.round(i);
    S.finish(h);
}

// The same with the scheduler fenced every 4 rounds: a message whose words
// are all known up front otherwise has its whole schedule (W[16..63] + K)
// hoisted ahead of the rounds, 64 live values; kernels that run many
// compressions back to back at 3 waves/SIMD (k_hkdf_key_setup) spilled them.
__device__ __forceinline__ void sha256_compress_fenced(uint32_t h[8], const uint32_t w[16]) {
    Sha256 S;
    S.start(h);
#pragma unroll
    for (int k = 0; k < 16; ++k) S.w[k] = w[k];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        S.round(i);
        if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
    S.finish(h);
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

// The last compressions of an HMAC through ONE inlined sha256_compress, so a
// kernel's packet loop carries a single copy of the 64 unrolled rounds:
// k = first..2 runs the full block `blk` (k = 0), the final padded block `fin`
// (k = 1) and the outer hash of the inner digest under the opad midstate
// (k = 2).  h: the inner state in, the tag out.
__device__ __forceinline__ void hmac_finish(uint32_t h[8], uint32_t first, const uint32_t blk[16],
                                            const uint32_t fin[16], const uint32_t opad[8]) {
#pragma nounroll
    for (uint32_t k = first; k < 3u; ++k) {
        uint32_t w[16];
        if (k == 2u) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                w[j] = h[j];
                h[j] = opad[j];
            }
            w[8] = 0x80000000u;
#pragma unroll
            for (int j = 9; j < 15; ++j) w[j] = 0u;
            w[15] = (64u + 32u) * 8u;
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) w[j] = k == 0u ? blk[j] : fin[j];
        }
        sha256_compress(h, w);
    }
}

// Final padded block of an HMAC inner hash: the first fu (0..3) 16-B units of
// u (big-endian words), 0x80, zeros, the 64-bit message length in bits.
__device__ __forceinline__ void sha_final_block(uint32_t fin[16], const uint32_t u[16], uint32_t fu, uint64_t bits) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
        fin[k] = (uint32_t)k < 4u * fu ? u[k] : ((uint32_t)k == 4u * fu ? 0x80000000u : 0u);
    fin[14] = (uint32_t)(bits >> 32);
    fin[15] = (uint32_t)bits;
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

// --------------------------------------------- interleaved AES + SHA quads --
//
// Four cipher blocks (one SHA-256 message block of 64 B) per call.  The
// SHA-256 rounds of an independent message block are spread one per AES round
// so the wave always has VALU work to issue while its LDS lookups are in
// flight: 4*NR AES rounds carry SHA rounds 0..4*NR-1, the rest follow.

// CBC encryption of x[0..3] chained from `chain` (serial), SHA rounds of S
// interleaved when WITH_SHA.
template <int NR, bool WITH_SHA>
__device__ __forceinline__ void enc_quad(u32x4 c[4], const u32x4 x[4], u32x4 chain, const uint32_t *rk,
                                         const Lanes &L, Sha256 &S) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const u32x4 in = x[b] ^ (b == 0 ? chain : c[b - 1]);
        uint32_t st[4] = {in.x ^ rk[0], in.y ^ rk[1], in.z ^ rk[2], in.w ^ rk[3]};
#pragma unroll
        for (int r = 1; r < NR; ++r) {
            uint32_t v[16];
            tround_load<false>(v, st, L);      // 16 LDS lookups in flight ...
            // ... while one SHA-256 round issues (a sched_barrier on either
            // side of it was 0.9-2.4 % slower on c2 decrypt and c3)
            if (WITH_SHA) S.round(b * NR + r - 1);
            tround_mix(st, v, rk + 4 * r);
        }
        const uint32_t s0 = st[0], s1 = st[1], s2 = st[2], s3 = st[3];
        c[b].x = tlast_enc(s0, s1, s2, s3, rk[4 * NR + 0], L);
        c[b].y = tlast_enc(s1, s2, s3, s0, rk[4 * NR + 1], L);
        c[b].z = tlast_enc(s2, s3, s0, s1, rk[4 * NR + 2], L);
        c[b].w = tlast_enc(s3, s0, s1, s2, rk[4 * NR + 3], L);
        if (WITH_SHA) S.round(b * NR + NR - 1);
    }
    if (WITH_SHA) {
#pragma unroll
        for (int i = 4 * NR; i < 64; ++i) S.round(i);
    }
}

// CBC decryption of c[0..3] (independent blocks, chained only by the XOR),
// equivalent inverse cipher with Td tables in regions 0/1:
// t_j = Td0[s_j.b0] ^ Td1[s_{j-1}.b1] ^ Td2[s_{j-2}.b2] ^ Td3[s_{j-3}.b3] ^ dk_j,
// SHA rounds of S interleaved when WITH_SHA.
template <int NR, bool WITH_SHA, bool SHIFT = false>
__device__ __forceinline__ void dec_quad(u32x4 p[4], const u32x4 c[4], u32x4 chain, const uint32_t *dk,
                                         const Lanes &L, Sha256 &S) {
    uint32_t s[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        s[b][0] = c[b].x ^ dk[0]; s[b][1] = c[b].y ^ dk[1]; s[b][2] = c[b].z ^ dk[2]; s[b][3] = c[b].w ^ dk[3];
    }
#pragma unroll
    for (int r = 1; r < NR; ++r) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t v[16];
            tround_load<true, SHIFT>(v, s[b], L);
            if (WITH_SHA) S.round((r - 1) * 4 + b);
            tround_mix(s[b], v, dk + 4 * r);
        }
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        u32x4 o;
        o.x = tlast_dec(s[b][0], s[b][3], s[b][2], s[b][1], dk[4 * NR + 0], L);
        o.y = tlast_dec(s[b][1], s[b][0], s[b][3], s[b][2], dk[4 * NR + 1], L);
        o.z = tlast_dec(s[b][2], s[b][1], s[b][0], s[b][3], dk[4 * NR + 2], L);
        o.w = tlast_dec(s[b][3], s[b][2], s[b][1], s[b][0], dk[4 * NR + 3], L);
        p[b] = o ^ (b == 0 ? chain : c[b - 1]);
        if (WITH_SHA) S.round(4 * (NR - 1) + b);
    }
    if (WITH_SHA) {
#pragma unroll
        for (int i = 4 * NR; i < 64; ++i) S.round(i);
    }
}

}  // namespace rnstok
