// bs_aes.h — bitsliced AES pieces for the bitsliced-CBC probe (tools/bs_probe.hip).
//
// Representation: a 32-bit word is one bit plane across 32 independent
// packets (bit j = packet j).  A lane holds one state column (4 rows x 8 bit
// planes = 32 words) of 32 packets; the quad of lanes 4g..4g+3 holds the 4
// columns, so ShiftRows is a DPP quad permute and MixColumns stays in the lane.
//
// The S-box is the Boyar-Peralta circuit (32 AND, 83 XOR/XNOR; "A depth-16
// circuit for the AES S-box", 2011) written out gate by gate; bs_selftest()
// checks it against the FIPS-197 S-box exhaustively.  Shared by host and
// device code.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define BS_FN __host__ __device__ __forceinline__
#else
#define BS_FN static inline
#endif

// q[k] = bit plane k of the byte (k = 0 is the least significant bit).
BS_FN void bs_sbox(uint32_t q[8]) {
    const uint32_t x0 = q[7], x1 = q[6], x2 = q[5], x3 = q[4], x4 = q[3], x5 = q[2], x6 = q[1], x7 = q[0];
    // top linear layer
    const uint32_t y14 = x3 ^ x5, y13 = x0 ^ x6, y9 = x0 ^ x3, y8 = x0 ^ x5, t0 = x1 ^ x2;
    const uint32_t y1 = t0 ^ x7, y4 = y1 ^ x3, y12 = y13 ^ y14, y2 = y1 ^ x0, y5 = y1 ^ x6;
    const uint32_t y3 = y5 ^ y8, t1 = x4 ^ y12, y15 = t1 ^ x5, y20 = t1 ^ x1, y6 = y15 ^ x7;
    const uint32_t y10 = y15 ^ t0, y11 = y20 ^ y9, y7 = x7 ^ y11, y17 = y10 ^ y11, y19 = y10 ^ y8;
    const uint32_t y16 = t0 ^ y11, y21 = y13 ^ y16, y18 = x0 ^ y16;
    // shared non-linear middle
    const uint32_t t2 = y12 & y15, t3 = y3 & y6, t4 = t3 ^ t2, t5 = y4 & x7, t6 = t5 ^ t2;
    const uint32_t t7 = y13 & y16, t8 = y5 & y1, t9 = t8 ^ t7, t10 = y2 & y7, t11 = t10 ^ t7;
    const uint32_t t12 = y9 & y11, t13 = y14 & y17, t14 = t13 ^ t12, t15 = y8 & y10, t16 = t15 ^ t12;
    const uint32_t t17 = t4 ^ t14, t18 = t6 ^ t16, t19 = t9 ^ t14, t20 = t11 ^ t16;
    const uint32_t t21 = t17 ^ y20, t22 = t18 ^ y19, t23 = t19 ^ y21, t24 = t20 ^ y18;
    const uint32_t t25 = t21 ^ t22, t26 = t21 & t23, t27 = t24 ^ t26, t28 = t25 & t27, t29 = t28 ^ t22;
    const uint32_t t30 = t23 ^ t24, t31 = t22 ^ t26, t32 = t31 & t30, t33 = t32 ^ t24, t34 = t23 ^ t33;
    const uint32_t t35 = t27 ^ t33, t36 = t24 & t35, t37 = t36 ^ t34, t38 = t27 ^ t36, t39 = t29 & t38;
    const uint32_t t40 = t25 ^ t39;
    const uint32_t t41 = t40 ^ t37, t42 = t29 ^ t33, t43 = t29 ^ t40, t44 = t33 ^ t37, t45 = t42 ^ t41;
    const uint32_t z0 = t44 & y15, z1 = t37 & y6, z2 = t33 & x7, z3 = t43 & y16, z4 = t40 & y1;
    const uint32_t z5 = t29 & y7, z6 = t42 & y11, z7 = t45 & y17, z8 = t41 & y10, z9 = t44 & y12;
    const uint32_t z10 = t37 & y3, z11 = t33 & y4, z12 = t43 & y13, z13 = t40 & y5, z14 = t29 & y2;
    const uint32_t z15 = t42 & y9, z16 = t45 & y14, z17 = t41 & y8;
    // bottom linear layer
    const uint32_t t46 = z15 ^ z16, t47 = z10 ^ z11, t48 = z5 ^ z13, t49 = z9 ^ z10, t50 = z2 ^ z12;
    const uint32_t t51 = z2 ^ z5, t52 = z7 ^ z8, t53 = z0 ^ z3, t54 = z6 ^ z7, t55 = z16 ^ z17;
    const uint32_t t56 = z12 ^ t48, t57 = t50 ^ t53, t58 = z4 ^ t46, t59 = z3 ^ t54, t60 = t46 ^ t57;
    const uint32_t t61 = z14 ^ t57, t62 = t52 ^ t58, t63 = t49 ^ t58, t64 = z4 ^ t59, t65 = t61 ^ t62;
    const uint32_t t66 = z1 ^ t63;
    const uint32_t s0 = t59 ^ t63, s6 = t56 ^ ~t62, s7 = t48 ^ ~t60, t67 = t64 ^ t65;
    const uint32_t s3 = t53 ^ t66, s4 = t51 ^ t66, s5 = t47 ^ t65, s1 = t64 ^ ~s3, s2 = t55 ^ ~t67;
    q[7] = s0; q[6] = s1; q[5] = s2; q[4] = s3; q[3] = s4; q[2] = s5; q[1] = s6; q[0] = s7;
}

// GF(2^8) doubling of one byte in planes: out = xtime(d).
BS_FN void bs_xtime(uint32_t o[8], const uint32_t d[8]) {
    o[0] = d[7]; o[1] = d[0] ^ d[7]; o[2] = d[1]; o[3] = d[2] ^ d[7];
    o[4] = d[3] ^ d[7]; o[5] = d[4]; o[6] = d[5]; o[7] = d[6];
}

// MixColumns + AddRoundKey of one column held in one lane: a[r][k] rows r,
// planes k; b_r = a_r ^ t ^ xtime(a_r ^ a_{r+1}) ^ rk_r, t = a0^a1^a2^a3.
BS_FN void bs_mix_ark(uint32_t a[4][8], const uint32_t rk[32]) {
    uint32_t t[8], o[4][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = a[0][k] ^ a[1][k] ^ a[2][k] ^ a[3][k];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        uint32_t d[8], x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = a[r][k] ^ a[(r + 1) & 3][k];
        bs_xtime(x, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[r][k] = a[r][k] ^ t[k] ^ x[k] ^ rk[8 * r + k];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 8; ++k) a[r][k] = o[r][k];
}

// 32x32 bit-matrix transpose in place: out[q] bit j = in[j] bit q.
// Self-inverse, so it also turns planes back into words.
BS_FN void bs_transpose(uint32_t w[32]) {
    uint32_t m = 0x0000FFFFu;
#pragma unroll
    for (int s = 16; s != 0; s >>= 1, m ^= (m << s)) {
#pragma unroll
        for (int k = 0; k < 32; k = (k + s + 1) & ~s) {
            // swap the high s-bit fields of w[k] with the low fields of w[k+s]
            const uint32_t t = ((w[k] >> s) ^ w[k + s]) & m;
            w[k + s] ^= t;
            w[k] ^= t << s;
        }
    }
}
