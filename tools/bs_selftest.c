// bs_selftest.c — host check of tools/bs_aes.h: the bitsliced S-box against the
// FIPS-197 S-box (all 256 inputs), the transpose, and a bitsliced AES-256 block
// encryption (32 packets x 4 columns emulating the lane quad) against the
// FIPS-197 C.3 known answer.   gcc -O2 -o /tmp/bs_selftest tools/bs_selftest.c && /tmp/bs_selftest
#include <stdio.h>
#include <string.h>

#include "bs_aes.h"

static uint8_t SB[256];

static uint8_t xt(uint8_t b) { return (uint8_t)((b << 1) ^ ((b & 0x80) ? 0x1b : 0)); }
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        a = xt(a);
        b >>= 1;
    }
    return p;
}
static void make_sbox(void) {
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        for (int y = 1; y < 256 && x; ++y)
            if (gmul((uint8_t)x, (uint8_t)y) == 1) inv = (uint8_t)y;
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; ++i) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        SB[x] = s ^ 0x63;
    }
}

// AES-256 key expansion, 60 words; word = bytes b0..b3 little-endian (b0 = row 0)
static void expand(const uint8_t key[32], uint32_t w[60]) {
    for (int i = 0; i < 8; ++i) w[i] = key[4 * i] | key[4 * i + 1] << 8 | key[4 * i + 2] << 16 | (uint32_t)key[4 * i + 3] << 24;
    uint8_t rc = 1;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = w[i - 1];
        if (i % 8 == 0) {
            t = (t >> 8) | (t << 24);
            t = SB[t & 255] | SB[(t >> 8) & 255] << 8 | SB[(t >> 16) & 255] << 16 | (uint32_t)SB[t >> 24] << 24;
            t ^= rc;
            rc = xt(rc);
        } else if (i % 8 == 4) {
            t = SB[t & 255] | SB[(t >> 8) & 255] << 8 | SB[(t >> 16) & 255] << 16 | (uint32_t)SB[t >> 24] << 24;
        }
        w[i] = w[i - 8] ^ t;
    }
}

int main(void) {
    make_sbox();
    // S-box, 8 groups of 32 inputs
    for (int g = 0; g < 8; ++g) {
        uint32_t q[8] = {0};
        for (int j = 0; j < 32; ++j)
            for (int k = 0; k < 8; ++k) q[k] |= (uint32_t)(((32 * g + j) >> k) & 1) << j;
        bs_sbox(q);
        for (int j = 0; j < 32; ++j) {
            int v = 0;
            for (int k = 0; k < 8; ++k) v |= ((q[k] >> j) & 1) << k;
            if (v != SB[32 * g + j]) {
                printf("sbox mismatch at %d: %02x vs %02x\n", 32 * g + j, v, SB[32 * g + j]);
                return 1;
            }
        }
    }
    printf("sbox ok\n");
    // transpose
    uint32_t w[32], o[32];
    for (int i = 0; i < 32; ++i) w[i] = o[i] = 0x9e3779b9u * (i + 1) ^ (0x85ebca6bu >> (i % 7));
    bs_transpose(w);
    for (int q = 0; q < 32; ++q)
        for (int j = 0; j < 32; ++j)
            if (((w[q] >> j) & 1) != ((o[j] >> q) & 1)) {
                printf("transpose mismatch %d %d\n", q, j);
                return 1;
            }
    bs_transpose(w);
    if (memcmp(w, o, sizeof w)) { printf("transpose not involutive\n"); return 1; }
    printf("transpose ok\n");
    // AES-256 FIPS-197 C.3, all 32 packets the same block; 4 "lanes" = columns
    uint8_t key[32], pt[16];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)i;
    for (int i = 0; i < 16; ++i) pt[i] = (uint8_t)(0x11 * i);
    const uint8_t expect[16] = {0x8e, 0xa2, 0xb7, 0xca, 0x51, 0x67, 0x45, 0xbf,
                                0xea, 0xfc, 0x49, 0x90, 0x4b, 0x49, 0x60, 0x89};
    uint32_t rkw[60];
    expand(key, rkw);
    uint32_t st[4][32];          // [column][plane 8r+k]
    for (int c = 0; c < 4; ++c) {
        uint32_t col = pt[4 * c] | pt[4 * c + 1] << 8 | pt[4 * c + 2] << 16 | (uint32_t)pt[4 * c + 3] << 24;
        for (int j = 0; j < 32; ++j) st[c][j] = col;
        bs_transpose(st[c]);
    }
    uint32_t rk[15][4][32];      // bitsliced round keys: plane mask 0 / ~0
    for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 4; ++c)
            for (int q = 0; q < 32; ++q) rk[r][c][q] = ((rkw[4 * r + c] >> q) & 1) ? 0xffffffffu : 0u;
    for (int c = 0; c < 4; ++c)
        for (int q = 0; q < 32; ++q) st[c][q] ^= rk[0][c][q];
    for (int r = 1; r <= 14; ++r) {
        uint32_t ns[4][32];
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row)          // ShiftRows: row from column c + row
                for (int k = 0; k < 8; ++k) ns[c][8 * row + k] = st[(c + row) & 3][8 * row + k];
        for (int c = 0; c < 4; ++c) {
            for (int row = 0; row < 4; ++row) bs_sbox(&ns[c][8 * row]);
            if (r < 14) {
                bs_mix_ark((uint32_t(*)[8])ns[c], rk[r][c]);
            } else {
                for (int q = 0; q < 32; ++q) ns[c][q] ^= rk[14][c][q];
            }
        }
        memcpy(st, ns, sizeof st);
    }
    for (int c = 0; c < 4; ++c) {
        bs_transpose(st[c]);
        for (int j = 0; j < 32; ++j)
            for (int b = 0; b < 4; ++b)
                if (((st[c][j] >> (8 * b)) & 255) != expect[4 * c + b]) {
                    printf("aes mismatch col %d packet %d byte %d\n", c, j, b);
                    return 1;
                }
    }
    printf("aes-256 kat ok\n");
    return 0;
}
