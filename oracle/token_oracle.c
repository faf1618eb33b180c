/*
 * oracle/token_oracle.c — CPU restatement of Reticulum's encrypted-token path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * kernels in reticulum_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never links,
 * imports or calls it.
 *
 * Parity is pinned by tests/golden/token_vectors.json, which tests/golden/gen_golden.py
 * produced by importing the reference RNS/Cryptography in the build
 * container (see tests/test_oracle.py).
 *
 * Written from FIPS-197 (AES), FIPS 180-4 (SHA-256), RFC 2104 (HMAC) and the
 * reference's token layout.  Reference call sites it follows (paths relative
 * to markqvist/Reticulum 1.4.2):
 *   Token key split        RNS/Cryptography/Token.py:58-74
 *   Token.encrypt          RNS/Cryptography/Token.py:87-97
 *   Token.verify_hmac      RNS/Cryptography/Token.py:77-84
 *   Token.decrypt          RNS/Cryptography/Token.py:100-114
 *   PKCS7 pad / unpad      RNS/Cryptography/PKCS7.py:35-39, 42-48
 *   AES-256 key expansion  RNS/Cryptography/aes/aes256.py:146-175
 *   AES block cipher       RNS/Cryptography/aes/aes256.py:177-213
 *   CBC chaining           RNS/Cryptography/aes/aes256.py:215-235
 *   AES-128 (32 B keys)    RNS/Cryptography/aes/aes128.py:156-326, AES.py:43-76
 *   HMAC (key pad, ipad/opad) RNS/Cryptography/HMAC.py:47-84,114-125
 *   HKDF-SHA256            RNS/Cryptography/HKDF.py:35-62 (oracle_hkdf)
 *   SHA-256                hashlib.sha256 (third-party: CPython _hashlib over
 *                          OpenSSL 3.0.2), restated from FIPS 180-4.
 *
 * Byte-oriented on purpose: it shares no table layout or code with the HIP
 * kernels it checks.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

/* Per-packet status codes (same values as include/rnstok.h). */
enum { ST_OK = 0, ST_TOO_SHORT = 1, ST_BAD_HMAC = 2, ST_BAD_CT_LEN = 3, ST_BAD_PAD = 4 };

/* ------------------------------------------------------------------ AES -- */

static uint8_t SBOX[256], INV_SBOX[256];
static int tables_ready = 0;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

/* S-box from its definition (FIPS-197 §5.1.1): multiplicative inverse in
 * GF(2^8) followed by the affine map. */
static void build_tables(void) {
    if (tables_ready) return;
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x) for (int y = 1; y < 256; ++y) if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; ++i) { r = (uint8_t)((r << 1) | (r >> 7)); s ^= r; }
        s ^= 0x63;
        SBOX[x] = s;
        INV_SBOX[s] = (uint8_t)x;
    }
    tables_ready = 1;
}

/* Key expansion (FIPS-197 §5.2) for Nk = 4 or 8 words.  rk holds 4*(Nr+1) words
 * as bytes, column-major like the reference's key matrices. */
static int expand_key(const uint8_t *key, int key_bytes, uint8_t rk[240]) {
    int nk = key_bytes / 4, nr = nk + 6, total = 4 * (nr + 1);
    uint8_t rcon = 1;
    memcpy(rk, key, (size_t)key_bytes);
    for (int i = nk; i < total; ++i) {
        uint8_t w[4];
        memcpy(w, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            uint8_t t = w[0];
            w[0] = SBOX[w[1]] ^ rcon; w[1] = SBOX[w[2]]; w[2] = SBOX[w[3]]; w[3] = SBOX[t];
            rcon = gf_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            for (int j = 0; j < 4; ++j) w[j] = SBOX[w[j]];
        }
        for (int j = 0; j < 4; ++j) rk[4 * i + j] = rk[4 * (i - nk) + j] ^ w[j];
    }
    return nr;
}

static void add_round_key(uint8_t s[16], const uint8_t *k) { for (int i = 0; i < 16; ++i) s[i] ^= k[i]; }

/* state byte index = 4*col + row */
static void sub_shift(uint8_t s[16]) {
    uint8_t t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) t[4 * c + r] = SBOX[s[4 * ((c + r) & 3) + r]];
    memcpy(s, t, 16);
}
static void inv_sub_shift(uint8_t s[16]) {
    uint8_t t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) t[4 * ((c + r) & 3) + r] = INV_SBOX[s[4 * c + r]];
    memcpy(s, t, 16);
}
static void mix(uint8_t s[16]) {
    for (int c = 0; c < 4; ++c) {
        uint8_t *a = s + 4 * c, b[4];
        for (int r = 0; r < 4; ++r)
            b[r] = gf_mul(a[r], 2) ^ gf_mul(a[(r + 1) & 3], 3) ^ a[(r + 2) & 3] ^ a[(r + 3) & 3];
        memcpy(a, b, 4);
    }
}
static void inv_mix(uint8_t s[16]) {
    for (int c = 0; c < 4; ++c) {
        uint8_t *a = s + 4 * c, b[4];
        for (int r = 0; r < 4; ++r)
            b[r] = gf_mul(a[r], 14) ^ gf_mul(a[(r + 1) & 3], 11) ^ gf_mul(a[(r + 2) & 3], 13) ^ gf_mul(a[(r + 3) & 3], 9);
        memcpy(a, b, 4);
    }
}
static void aes_encrypt_block(const uint8_t *rk, int nr, uint8_t s[16]) {
    add_round_key(s, rk);
    for (int r = 1; r < nr; ++r) { sub_shift(s); mix(s); add_round_key(s, rk + 16 * r); }
    sub_shift(s); add_round_key(s, rk + 16 * nr);
}
static void aes_decrypt_block(const uint8_t *rk, int nr, uint8_t s[16]) {
    add_round_key(s, rk + 16 * nr);
    for (int r = nr - 1; r > 0; --r) { inv_sub_shift(s); add_round_key(s, rk + 16 * r); inv_mix(s); }
    inv_sub_shift(s); add_round_key(s, rk);
}

/* -------------------------------------------------------------- SHA-256 -- */

typedef struct { uint32_t h[8]; uint8_t buf[64]; uint64_t len; } sha256_ctx;

static const uint32_t K256[64] = {
    0x428a2f98,0x71374491,0xb5c0fbcf,0xe9b5dba5,0x3956c25b,0x59f111f1,0x923f82a4,0xab1c5ed5,
    0xd807aa98,0x12835b01,0x243185be,0x550c7dc3,0x72be5d74,0x80deb1fe,0x9bdc06a7,0xc19bf174,
    0xe49b69c1,0xefbe4786,0x0fc19dc6,0x240ca1cc,0x2de92c6f,0x4a7484aa,0x5cb0a9dc,0x76f988da,
    0x983e5152,0xa831c66d,0xb00327c8,0xbf597fc7,0xc6e00bf3,0xd5a79147,0x06ca6351,0x14292967,
    0x27b70a85,0x2e1b2138,0x4d2c6dfc,0x53380d13,0x650a7354,0x766a0abb,0x81c2c92e,0x92722c85,
    0xa2bfe8a1,0xa81a664b,0xc24b8b70,0xc76c51a3,0xd192e819,0xd6990624,0xf40e3585,0x106aa070,
    0x19a4c116,0x1e376c08,0x2748774c,0x34b0bcb5,0x391c0cb3,0x4ed8aa4a,0x5b9cca4f,0x682e6ff3,
    0x748f82ee,0x78a5636f,0x84c87814,0x8cc70208,0x90befffa,0xa4506ceb,0xbef9a3f7,0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_compress(uint32_t h[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha256_init(sha256_ctx *c) {
    static const uint32_t iv[8] = {0x6a09e667,0xbb67ae85,0x3c6ef372,0xa54ff53a,0x510e527f,0x9b05688c,0x1f83d9ab,0x5be0cd19};
    memcpy(c->h, iv, sizeof iv);
    c->len = 0;
}
static void sha256_update(sha256_ctx *c, const uint8_t *p, size_t n) {
    while (n) {
        size_t used = (size_t)(c->len & 63), take = 64 - used;
        if (take > n) take = n;
        memcpy(c->buf + used, p, take);
        c->len += take; p += take; n -= take;
        if ((c->len & 63) == 0) sha256_compress(c->h, c->buf);
    }
}
static void sha256_final(sha256_ctx *c, uint8_t out[32]) {
    uint64_t bits = c->len * 8;
    uint8_t pad = 0x80, z = 0, lenb[8];
    sha256_update(c, &pad, 1);
    while ((c->len & 63) != 56) sha256_update(c, &z, 1);
    for (int i = 0; i < 8; ++i) lenb[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha256_update(c, lenb, 8);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(c->h[i] >> 24); out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->h[i] >> 8); out[4 * i + 3] = (uint8_t)c->h[i];
    }
}

void oracle_sha256(const uint8_t *msg, uint64_t n, uint8_t out[32]) {
    sha256_ctx c; sha256_init(&c); sha256_update(&c, msg, (size_t)n); sha256_final(&c, out);
}

/* RFC 2104 with SHA-256; keys longer than the 64-byte block are hashed first,
 * shorter ones zero-padded (HMAC.py:73-82). */
void oracle_hmac_sha256(const uint8_t *key, uint32_t klen, const uint8_t *msg, uint64_t n, uint8_t out[32]) {
    uint8_t k[64] = {0}, ip[64], op[64], inner[32];
    if (klen > 64) oracle_sha256(key, klen, k); else memcpy(k, key, klen);
    for (int i = 0; i < 64; ++i) { ip[i] = k[i] ^ 0x36; op[i] = k[i] ^ 0x5c; }
    sha256_ctx c;
    sha256_init(&c); sha256_update(&c, ip, 64); sha256_update(&c, msg, (size_t)n); sha256_final(&c, inner);
    sha256_init(&c); sha256_update(&c, op, 64); sha256_update(&c, inner, 32); sha256_final(&c, out);
}

/* ---------------------------------------------------------------- token -- */

/* Token key split (Token.py:61-72): 64 B -> sk = key[0:32], ek = key[32:64]
 * (AES-256-CBC); 32 B -> sk = key[0:16], ek = key[16:32] (AES-128-CBC). */
static int split_key(const uint8_t *key, uint32_t klen, const uint8_t **sk, uint32_t *sklen, const uint8_t **ek) {
    if (klen != 64 && klen != 32) return -1;
    *sklen = klen / 2; *sk = key; *ek = key + klen / 2;
    return 0;
}

uint64_t oracle_token_len(uint32_t pt_len) { return 16u + 16u * ((uint64_t)pt_len / 16 + 1) + 32u; }

/* Token.encrypt (Token.py:87-97): iv || AES-CBC(ek, iv, PKCS7(pt)) || HMAC(sk, iv||ct).
 * Returns the token length, or -1 for an invalid key. */
int64_t oracle_token_encrypt(const uint8_t *key, uint32_t klen, const uint8_t iv[16],
                             const uint8_t *pt, uint32_t L, uint8_t *tok) {
    const uint8_t *sk, *ek; uint32_t sklen;
    uint8_t rk[240];
    build_tables();
    if (split_key(key, klen, &sk, &sklen, &ek)) return -1;
    int nr = expand_key(ek, (int)(klen / 2), rk);
    uint32_t nb = L / 16 + 1, padv = 16 - L % 16;       /* PKCS7.pad, PKCS7.py:35-39 */
    uint8_t prev[16];
    memcpy(tok, iv, 16);
    memcpy(prev, iv, 16);
    for (uint32_t b = 0; b < nb; ++b) {
        uint8_t s[16];
        for (int i = 0; i < 16; ++i) {
            uint32_t idx = 16 * b + (uint32_t)i;
            uint8_t p = idx < L ? pt[idx] : (uint8_t)padv;
            s[i] = p ^ prev[i];                          /* CBC, aes256.py:219-222 */
        }
        aes_encrypt_block(rk, nr, s);
        memcpy(tok + 16 + 16 * b, s, 16);
        memcpy(prev, s, 16);
    }
    uint64_t signed_len = 16 + 16 * (uint64_t)nb;
    oracle_hmac_sha256(sk, sklen, tok, signed_len, tok + signed_len);
    return (int64_t)(signed_len + 32);
}

/* Token.decrypt (Token.py:100-114) with the reference's error order:
 * len <= 32 -> TOO_SHORT (Token.py:78); tag mismatch -> BAD_HMAC (:102);
 * iv shorter than 16, empty ct or ct % 16 != 0 -> BAD_CT_LEN (aes256.py:136,
 * 227; PKCS7.py:44 IndexError on empty data); last byte > 16 -> BAD_PAD
 * (PKCS7.py:45-46).  Unpad is lenient: n = 0 and unchecked pad bytes pass.
 * pt receives max(T-48, 0) bytes; *pt_len the unpadded length on success. */
int oracle_token_decrypt(const uint8_t *key, uint32_t klen, const uint8_t *tok, uint64_t T,
                         uint8_t *pt, uint64_t *pt_len) {
    const uint8_t *sk, *ek; uint32_t sklen;
    uint8_t rk[240], tag[32];
    build_tables();
    *pt_len = 0;
    if (split_key(key, klen, &sk, &sklen, &ek)) return -1;
    if (T <= 32) return ST_TOO_SHORT;
    oracle_hmac_sha256(sk, sklen, tok, T - 32, tag);
    if (memcmp(tag, tok + T - 32, 32) != 0) return ST_BAD_HMAC;
    if (T < 48) return ST_BAD_CT_LEN;
    uint64_t ct_len = T - 48;
    if (ct_len == 0 || ct_len % 16 != 0) return ST_BAD_CT_LEN;
    int nr = expand_key(ek, (int)(klen / 2), rk);
    const uint8_t *prev = tok;
    for (uint64_t b = 0; b < ct_len / 16; ++b) {
        uint8_t s[16];
        memcpy(s, tok + 16 + 16 * b, 16);
        aes_decrypt_block(rk, nr, s);
        for (int i = 0; i < 16; ++i) pt[16 * b + i] = s[i] ^ prev[i];   /* aes256.py:230-232 */
        prev = tok + 16 + 16 * b;
    }
    uint8_t n = pt[ct_len - 1];
    if (n > 16) return ST_BAD_PAD;
    *pt_len = ct_len - n;
    return ST_OK;
}

/* ----------------------------------------------------- batch (C-ABI mirror) --
 * Same argument meaning as rt_encrypt / rt_decrypt in include/rnstok.h, but
 * over host buffers, with keys given raw (n_keys x key_len bytes). */

typedef struct {
    const uint8_t *keys; uint32_t klen;
    const uint8_t *in; const uint64_t *in_off; const uint32_t *in_len;
    const uint32_t *key_idx; const uint8_t *iv;
    uint8_t *out; const uint64_t *out_off; uint32_t *out_len; int32_t *status;
    uint64_t lo, hi; int dec;
} job_t;

static void *run_job(void *arg) {
    job_t *j = (job_t *)arg;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint8_t *k = j->keys + (uint64_t)(j->key_idx ? j->key_idx[i] : 0) * j->klen;
        if (!j->dec) {
            oracle_token_encrypt(k, j->klen, j->iv + 16 * i, j->in + j->in_off[i], j->in_len[i], j->out + j->out_off[i]);
        } else {
            uint64_t pl = 0;
            int st = oracle_token_decrypt(k, j->klen, j->in + j->in_off[i], j->in_len[i], j->out + j->out_off[i], &pl);
            j->status[i] = st;
            j->out_len[i] = (uint32_t)pl;
        }
    }
    return NULL;
}

static int run_batch(job_t proto, uint64_t n, int threads) {
    build_tables();
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256]; job_t jobs[256]; int created[256] = {0};
    uint64_t per = (n + (uint64_t)threads - 1) / (uint64_t)threads;
    for (int t = 0; t < threads; ++t) {
        jobs[t] = proto;
        jobs[t].lo = per * (uint64_t)t; jobs[t].hi = jobs[t].lo + per;
        if (jobs[t].lo > n) jobs[t].lo = n;
        if (jobs[t].hi > n) jobs[t].hi = n;
        if (t > 0) created[t] = pthread_create(&tid[t], NULL, run_job, &jobs[t]) == 0;
    }
    run_job(&jobs[0]);
    for (int t = 1; t < threads; ++t) {
        if (created[t]) pthread_join(tid[t], NULL);
        else run_job(&jobs[t]);
    }
    return 0;
}

int oracle_encrypt_batch(const uint8_t *keys, uint32_t klen, const uint8_t *pt, const uint64_t *pt_off,
                         const uint32_t *pt_len, const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok,
                         const uint64_t *tok_off, uint64_t n, int threads) {
    if (klen != 32 && klen != 64) return -1;
    job_t j = {keys, klen, pt, pt_off, pt_len, key_idx, iv, tok, tok_off, NULL, NULL, 0, 0, 0};
    return run_batch(j, n, threads);
}

int oracle_decrypt_batch(const uint8_t *keys, uint32_t klen, const uint8_t *tok, const uint64_t *tok_off,
                         const uint32_t *tok_len, const uint32_t *key_idx, uint8_t *pt, const uint64_t *pt_off,
                         uint32_t *pt_len, int32_t *status, uint64_t n, int threads) {
    if (klen != 32 && klen != 64) return -1;
    job_t j = {keys, klen, tok, tok_off, tok_len, key_idx, NULL, pt, pt_off, pt_len, status, 0, 0, 1};
    return run_batch(j, n, threads);
}

/* Block-level hooks for unit tests of the restatement itself. */
void oracle_aes_encrypt_block(const uint8_t *key, uint32_t klen, const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[240]; build_tables();
    int nr = expand_key(key, (int)klen, rk);
    memcpy(out, in, 16); aes_encrypt_block(rk, nr, out);
}
void oracle_aes_decrypt_block(const uint8_t *key, uint32_t klen, const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[240]; build_tables();
    int nr = expand_key(key, (int)klen, rk);
    memcpy(out, in, 16); aes_decrypt_block(rk, nr, out);
}
void oracle_sbox(uint8_t out[256]) { build_tables(); memcpy(out, SBOX, 256); }

/* HKDF-SHA256 as RNS/Cryptography/HKDF.py:35-62 computes it:
 *   salt NULL or empty -> 32 zero bytes (:45-46); context NULL -> b"" (:48-49)
 *   PRK = HMAC(salt, ikm) (:51); T_i = HMAC(PRK, T_{i-1} || context || (i % 256)) (:56-60)
 *   output = (T_1 || T_2 || ...)[:length] (:62)
 * The argument checks (:40-44) belong to the caller (length >= 1, ikm given). */
void oracle_hkdf(const uint8_t *ikm, uint64_t ikm_len, const uint8_t *salt, uint32_t salt_len,
                 const uint8_t *context, uint32_t context_len, uint64_t length, uint8_t *out) {
    static const uint8_t zeros[32] = {0};
    if (!salt || salt_len == 0) { salt = zeros; salt_len = 32; }
    uint8_t prk[32], t[32];
    oracle_hmac_sha256(salt, salt_len, ikm, ikm_len, prk);
    uint8_t *msg = (uint8_t *)malloc(32 + (size_t)context_len + 1);
    uint64_t done = 0;
    for (uint64_t i = 0; done < length; ++i) {
        size_t m = 0;
        if (i) { memcpy(msg, t, 32); m = 32; }
        if (context_len) memcpy(msg + m, context, context_len);
        m += context_len;
        msg[m++] = (uint8_t)((i + 1) % 256);
        oracle_hmac_sha256(prk, 32, msg, m, t);
        uint64_t take = length - done < 32 ? length - done : 32;
        memcpy(out + done, t, take);
        done += take;
    }
    free(msg);
}
